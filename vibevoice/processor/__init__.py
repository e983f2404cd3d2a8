"""vibevoice.processor (reference path) -> vibevoice_amd.processor."""
