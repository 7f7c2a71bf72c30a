"""ORACLE package -- test infrastructure only (see oracle/oracle.py header)."""
