"""Algorithms: NMF engine, refits, consensus, OLS, gene statistics, Harmony."""
