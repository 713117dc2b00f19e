"""TEST INFRASTRUCTURE ONLY — CPU oracle for the bilateral-filter family.

Import only from tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.
"""
