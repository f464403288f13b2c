"""Drop-in replacement for the reference's `utils` package (format producers, test gate)."""
