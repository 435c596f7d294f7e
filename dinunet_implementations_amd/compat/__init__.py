"""COINSTAC compatibility: entry/local/remote callbacks over a file transport + simulator."""
