"""delta_crdt_ex_amd — MI355X-native batched delta-join and anti-entropy engine for
DeltaCrdt.AWLWWMap (reference: burmajam/delta_crdt_ex 0.5.10).

The product is the C-ABI library libdeltagpu (include/deltagpu.h, HIP kernels in
csrc/); this package builds it (`build.py`), binds it (`_abi.py`), keeps dot stores
device-resident (`store.py`), mirrors the reference's AWLWWMap module on top of it
(`aw_lww_map.py`), and generates the benchmark workloads (`workloads.py`).
"""
__version__ = "0.1.0"
