"""vibevoice.modular (reference path) -> vibevoice_amd."""
