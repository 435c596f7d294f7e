"""Task plugins (FS-Classification, ICA-Classification) and registries."""
