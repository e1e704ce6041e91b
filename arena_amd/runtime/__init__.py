"""Runtime services: job monitor, rendezvous helpers."""
