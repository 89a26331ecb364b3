"""TEST INFRASTRUCTURE ONLY: the CPU restatement (oracle) of Demikernel's receive path.

Importable by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg only — never by the product package
(demikernel_amd/), which has no CPU fallback. See oracle/dk_oracle.cpp for the restated reference lines and for how
the oracle is pinned (DESIGN.md "Oracle and parity").
"""
