"""COINSTAC container entry point (reference ``entry.py``): serve the site and remote callbacks."""
import local
import remote
from dinunet_implementations_amd.compat.coinstac import start

if __name__ == "__main__":
    start(local.run, remote.run)
