"""ORACLE — CPU restatement of the reference's hot path (test infrastructure only).

Importable only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
