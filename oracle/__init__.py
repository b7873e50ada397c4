"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the ov3d hot path.

Importable only from tests/, __graft_entry__.smoke() and bench.py's
cpu_baseline leg.  Never imported by the product package.
"""
