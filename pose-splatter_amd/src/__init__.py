"""Drop-in package mirroring the reference import path ``src.gaussian_renderer``."""
