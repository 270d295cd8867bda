"""Drop-in mirror of ``src.contrastor``."""
