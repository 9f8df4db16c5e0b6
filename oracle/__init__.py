"""Parity oracle — TEST INFRASTRUCTURE ONLY (see oracle/README.md).

Importable by `tests/`, `__graft_entry__.smoke()` and `bench.py`'s cpu_baseline leg only.
"""
