__version__ = "1.7.0+mi355x.r1"
