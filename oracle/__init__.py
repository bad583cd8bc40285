"""ORACLE package — test infrastructure only (see mrg_oracle.py header)."""
