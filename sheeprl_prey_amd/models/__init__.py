"""Shared network building blocks (reference ``sheeprl/models/models.py``): MLP, CNN / DeCNN stacks,
NatureCNN, the LayerNorm GRU cell and the multi-key encoder / decoder containers (``models.py``), plus the
batched critic ensembles (``ensemble.py``) used by SAC, DroQ and SAC-AE."""
from sheeprl_prey_amd.models.models import CNN, MLP, DeCNN, LayerNormGRUCell, MultiDecoder, MultiEncoder, NatureCNN

__all__ = ["MLP", "CNN", "DeCNN", "NatureCNN", "LayerNormGRUCell", "MultiEncoder", "MultiDecoder"]
