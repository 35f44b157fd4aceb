"""recommendsystem_amd — MI355X-native (gfx950 HIP) CTR feature-interaction training path of
yueshifeng/recommendSystem: embedding lookup + concat, AutoInt InteractingLayer, DIN pools and
MLP towers behind the reference's layer/model signatures.  See DESIGN.md.

All compute runs in librecsys_amd.so (C ABI: include/recsys_amd.h); there is no CPU fallback.
"""
from .embedding import (EmbeddingFeatures, SequenceEmbedding, SparseAdaGrad, SparseAdam,  # noqa: F401
                        SparseTable)
from .din import DIN, StaytimeDIN  # noqa: F401
from .layers import Dense, InteractingLayer, MultiLayerDense  # noqa: F401
from .autoint import AutoInt, AutoIntConfig, AutoIntTrainer, cross_entropy  # noqa: F401

__version__ = "0.1.0"
