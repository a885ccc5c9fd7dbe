"""Test-infrastructure oracle package (see oracle/oracle.py header)."""
