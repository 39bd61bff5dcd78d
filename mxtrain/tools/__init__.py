"""Operator tooling: image references, node bring-up, data staging."""
