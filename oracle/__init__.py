"""TEST INFRASTRUCTURE ONLY: CPU oracle (PCL-1.8 restatement) for the RANSAC plane path.

Importable only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
