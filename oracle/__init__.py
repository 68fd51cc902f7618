"""ORACLE — test infrastructure only.

A plain PyTorch-CPU restatement of the HL-HGAT hot path (deepika090/HL-HGAT,
lib/Hodge_Cheb_Conv.py, lib/Hodge_Dataset.py, lib/Hodge_ST_Model.py), each
function citing the reference line it follows.  It is the checker for the HIP
product path and the timed "reference CPU path" (cpu_baseline.kind = "port").

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this package; the product (hl-hgat_amd/hlhgat) never does.

Parity pinning: this restatement is checked against golden vectors produced by
running the reference's own class bodies (imported from /root/reference behind
a stand-in for the absent PyG/torch_scatter packages, see
tests/golden/make_golden.py) in tests/test_oracle_golden.py.
"""
