"""Developer tools (reference ``dev-scripts/``)."""
