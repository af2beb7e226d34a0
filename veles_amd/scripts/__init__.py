"""Console scripts (reference veles/scripts/)."""
