"""The head class the peptides-func training script defines for itself
(main_pepfunc_HL_HGCNN_dense_int3_attpool.py:36-168; BASELINE config 4).

It shadows lib/Hodge_ST_Model.py's class of the same name in that script
(NEAtt after EVERY level on the dense concatenation, l=0.5, sigmoid; K=1
initial convs; degree + 1e-6), so hlhgat keeps the two apart:
``hlhgat.hodge_st_model.HL_HGCNN_pepfunc_dense_int3_attpool`` is the library's,
this module's (also exported as ``hlhgat.HL_HGCNN_pepfunc_dense_int3_attpool``)
is the script's.
"""
from __future__ import annotations

from .hodge_st_model import _AttPoolHead

__all__ = ["HL_HGCNN_pepfunc_dense_int3_attpool"]


class HL_HGCNN_pepfunc_dense_int3_attpool(_AttPoolHead):
    """main_pepfunc_HL_HGCNN_dense_int3_attpool.py:36-168."""

    def __init__(self, channels=[2, 2, 2, 2], filters=[64, 128, 256, 512], mlp_channels=[],
                 K=2, node_dim=9, edge_dim=3, num_classes=10, dropout_ratio=0.0,
                 dropout_ratio_mlp=0.0, pool_loc=0, keig=20):
        super().__init__(channels, filters, mlp_channels, K, node_dim, edge_dim, num_classes,
                         dropout_ratio, dropout_ratio_mlp, pool_loc, keig, 0.5,
                         att_mode="every")

    def forward(self, datas, device="cuda:0", if_att=False, if_final_layer=False):
        # the pepfunc script orders the flags (if_att, if_final_layer) (:103)
        return super().forward(datas, device, if_final_layer=if_final_layer, if_att=if_att)
