"""L1: the `arena` command line."""
