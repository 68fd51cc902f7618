"""hlhgat — MI355X-native (gfx950) Hodge-Laplacian message passing for HL-HGAT.

Drop-in for the hot path of deepika090/HL-HGAT (lib/Hodge_Cheb_Conv.py):
HodgeLaguerreConv / HodgeChebConv / NodeEdgeInt / MSI / HL_filter / SAPool
keep the reference's constructors, forward signatures and state_dict keys; the
arithmetic runs in hand-written HIP kernels behind the C-ABI of
include/hlhgat.h (libhlhgat.so).  There is no CPU fallback: importing this
package loads the HIP library or raises.
"""
import os as _os

# Captured training steps are two chains of kernels (the HL blocks' node and
# edge chains): run a hipGraph on two hardware queues, not the runtime's
# default four, which adds cross-queue dependencies (same-box sweep: 2.74 ->
# 2.68 ms per config-2 step).  Read when HIP initialises; a
# value set by the user wins.
_os.environ.setdefault("DEBUG_HIP_FORCE_GRAPH_QUEUES", "2")

from . import ops  # noqa: F401,E402  (loads libhlhgat.so; raises if missing)
from .hodge_cheb_conv import (HL_filter, HodgeChebConv, HodgeLaguerreConv,  # noqa: F401,E402
                              HodgeLaguerreFastConv, MSI, NodeEdgeInt, SAPool)
from .hodge_dataset import (Batch, BoundaryOperator, PairData, adj2par1, collate,  # noqa: F401,E402
                            degree)
from .hodge_st_model import (HL_HGCNN_CIFAR10SP_dense_int3_attpool,  # noqa: F401,E402
                             HL_HGCNN_pepfunc_dense_int3_attpool, HL_HGCNN_TSP_dense_int3_pyr,
                             HL_HGCNN_zinc_dense_int3_pyr)
from .nn import BatchNorm, Linear, Sequential, global_mean_pool  # noqa: F401,E402

__version__ = "0.1.0"
