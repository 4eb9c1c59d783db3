"""Import-compatible mirror of the reference's `src.core` hot-path API."""
