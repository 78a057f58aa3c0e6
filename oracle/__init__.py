"""TEST INFRASTRUCTURE ONLY: CPU restatements of the reference's sampling path.
Imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only."""
