"""I/O, AnnData container, RNG twin, timing, plotting, synthetic data."""
