"""Parity checker for the MI355X CRC32C engine -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package.  The product path (foundationdb_amd/) never imports it.
"""
