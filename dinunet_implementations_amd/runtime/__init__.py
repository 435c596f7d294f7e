"""Site runtime: training step, trainer loop, site/fold orchestration."""
