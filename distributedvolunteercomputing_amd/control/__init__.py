"""control subpackage."""
