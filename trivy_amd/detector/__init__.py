"""Mirrors of the reference detector packages (pkg/detector/...)."""
