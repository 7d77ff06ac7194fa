"""Command-line data tools (``python -m rocfm.tools.<name>``)."""
