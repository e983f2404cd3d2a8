"""vibevoice.schedule (reference path) -> vibevoice_amd.schedule."""
