"""TEST INFRASTRUCTURE: the CPU oracle (see oracle/rtw_oracle.h).  Only tests/,
__graft_entry__.smoke() and bench.py's cpu_baseline leg may import this package."""
