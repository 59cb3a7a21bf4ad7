"""ORACLE — TEST INFRASTRUCTURE ONLY.  CPU restatement of the reference's
tree-hash path; importable only by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg.  The product (prysm_amd/) never imports it."""
