from sheeprl_prey_amd.models.models import CNN, MLP, DeCNN, LayerNormGRUCell, MultiDecoder, MultiEncoder, NatureCNN

__all__ = ["MLP", "CNN", "DeCNN", "NatureCNN", "LayerNormGRUCell", "MultiEncoder", "MultiDecoder"]
