"""End-to-end test of the operator on real processes: the reference's tests/scripts/end-to-end.sh
flow against an in-process API server, the operator as its own process and a kubelet that runs
the node's pods as processes (harness.py, kubelet.py)."""
