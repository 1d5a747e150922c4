"""graphlearninglayer_amd -- MI355X-native Graph Learning Layer hot path.

Drop-in for /root/reference/GLL.py: `from graphlearninglayer_amd import GLL` (or
`from graphlearninglayer_amd.GLL import LaplaceLearningSparseHard, knn_sym_dist,
stable_conjgrad`).  Kernels live in libgll.so (csrc/, C ABI in include/gll.h).
"""
from . import GLL  # noqa: F401
from .GLL import LaplaceLearningSparseHard, knn_sym_dist, stable_conjgrad  # noqa: F401
from .parallel import gather_predictions, shard_rank_seed  # noqa: F401

__all__ = ["GLL", "LaplaceLearningSparseHard", "knn_sym_dist", "stable_conjgrad",
           "gather_predictions", "shard_rank_seed"]
