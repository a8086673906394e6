"""Interactive command-line interface."""
