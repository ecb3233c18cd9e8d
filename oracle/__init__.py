"""ORACLE package — test infrastructure only (see decagon_oracle.py header).

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only.
"""
