"""Site datasets, splits and HBM-resident loaders."""
