"""jobs subpackage."""
