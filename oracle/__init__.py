"""TEST INFRASTRUCTURE ONLY: the CPU oracle (ort_oracle.c) and the reference-builder driver.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package.
"""
