"""Test infrastructure: CPU oracle for the DSTAGNN block hot path.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this
package.  The product package dstagnn_drought_amd never does.
"""
