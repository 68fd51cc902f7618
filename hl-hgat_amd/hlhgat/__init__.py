"""hlhgat — MI355X-native (gfx950) Hodge-Laplacian message passing for HL-HGAT.

Drop-in for the hot path of deepika090/HL-HGAT (lib/Hodge_Cheb_Conv.py):
HodgeLaguerreConv / HodgeChebConv / NodeEdgeInt / MSI / HL_filter / SAPool
keep the reference's constructors, forward signatures and state_dict keys; the
arithmetic runs in hand-written HIP kernels behind the C-ABI of
include/hlhgat.h (libhlhgat.so).  There is no CPU fallback: importing this
package loads the HIP library or raises.
"""
from . import ops  # noqa: F401,E402  (loads libhlhgat.so; raises if missing)
from .hodge_cheb_conv import (HL_filter, HodgeChebConv, HodgeLaguerreConv,  # noqa: F401,E402
                              HodgeLaguerreFastConv, MSI, NodeEdgeInt, SAPool)
from .hodge_dataset import (Batch, BoundaryOperator, PairData, adj2par1, collate,  # noqa: F401,E402
                            degree)
from .hodge_st_model import (HL_HGCNN_CIFAR10SP_dense_int3_attpool,  # noqa: F401,E402
                             HL_HGCNN_CIFAR10SP_dense_int3_pyr, HL_HGCNN_pepfunc_dense_int3_pyr,
                             HL_HGCNN_TSP_dense_int3_pyr, HL_HGCNN_zinc_dense_int3_attpool,
                             HL_HGCNN_zinc_dense_int3_pyr, HL_HGCNN_zinc_dense_poolint3_pyr)
# the peptides training script's own head (BASELINE config 4), which shadows
# the library class of that name there (hodge_st_model's)
from .main_pepfunc import HL_HGCNN_pepfunc_dense_int3_attpool  # noqa: F401,E402
from .nn import BatchNorm, Linear, Sequential, global_mean_pool  # noqa: F401,E402

__version__ = "0.1.0"
