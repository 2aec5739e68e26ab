"""Layer-construction helpers (reference: ``sheeprl/utils/model.py:12-235``) plus the fusion pass
that turns ``LayerNorm -> activation`` pairs into one fused HIP kernel."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Sequence, Tuple, Type, Union

import torch
from torch import Tensor, nn

from sheeprl_prey_amd import ops

ModuleType = Optional[Type[nn.Module]]
ArgType = Union[Tuple[Any, ...], Dict[Any, Any], None]
ArgsType = Union[ArgType, List[ArgType]]


def create_layer_with_args(layer_type: ModuleType, layer_args: Optional[ArgType]) -> nn.Module:
    if layer_type is None:
        raise ValueError("`layer_type` must be not None")
    if isinstance(layer_args, tuple):
        return layer_type(*layer_args)
    if isinstance(layer_args, dict):
        return layer_type(**layer_args)
    if layer_args is None:
        return layer_type()
    raise ValueError(f"`layer_args` must be None, tuple or dict, got {type(layer_args)}")


def miniblock(
    input_size: int,
    output_size: int,
    layer_type: Type[nn.Module] = nn.Linear,
    layer_args: ArgType = None,
    dropout_layer: ModuleType = None,
    dropout_args: ArgType = None,
    norm_layer: ModuleType = None,
    norm_args: ArgType = None,
    activation: ModuleType = None,
    act_args: ArgType = None,
) -> List[nn.Module]:
    """``layer -> [dropout] -> [norm] -> [activation]``."""
    if layer_args is None:
        layers: List[nn.Module] = [layer_type(input_size, output_size)]
    elif isinstance(layer_args, tuple):
        layers = [layer_type(input_size, output_size, *layer_args)]
    elif isinstance(layer_args, dict):
        layers = [layer_type(input_size, output_size, **layer_args)]
    else:
        raise ValueError(f"layer_args must be None, tuple or dict, got {type(layer_args)}")
    if dropout_layer is not None:
        layers.append(create_layer_with_args(dropout_layer, dropout_args))
    if norm_layer is not None:
        layers.append(create_layer_with_args(norm_layer, norm_args))
    if activation is not None:
        layers.append(create_layer_with_args(activation, act_args))
    return layers


def create_layers(
    layer_type: Union[ModuleType, List[ModuleType]], layer_args: Optional[ArgsType], num_layers: int
) -> Tuple[List[ModuleType], ArgsType]:
    if layer_type is None:
        return [None] * num_layers, [None] * num_layers
    if isinstance(layer_type, list):
        assert len(layer_type) == num_layers
        if isinstance(layer_args, list):
            assert len(layer_args) == num_layers
            return layer_type, layer_args
        return layer_type, [layer_args for _ in range(num_layers)]
    return [layer_type for _ in range(num_layers)], [layer_args for _ in range(num_layers)]


def per_layer_ortho_init_weights(module: nn.Module, gain: float = 1.0, bias: float = 0.0) -> None:
    if isinstance(module, nn.Linear):
        nn.init.orthogonal_(module.weight, gain=gain)
        if module.bias is not None:
            module.bias.data.fill_(bias)
    elif isinstance(module, nn.LSTM):
        for name, param in module.named_parameters():
            if "bias" in name:
                nn.init.constant_(param, val=bias)
            elif "weight" in name:
                nn.init.orthogonal_(param, gain=gain)
    elif isinstance(module, (nn.Sequential, nn.ModuleList)):
        for m in module:
            per_layer_ortho_init_weights(m, gain=gain, bias=bias)


def cnn_forward(model: nn.Module, input: Tensor, input_dim, output_dim) -> Tensor:
    """Flatten the leading dims before a CNN and restore them after."""
    batch_shapes = input.shape[: -len(input_dim)]
    flatten_input = input.reshape(-1, *input_dim)
    model_out = model(flatten_input)
    return model_out.reshape(*batch_shapes, *output_dim)


_ACT_NAMES = {nn.SiLU: "silu", nn.ELU: "elu", nn.ReLU: "relu", nn.Tanh: "tanh"}


class LayerNorm(nn.LayerNorm):
    """``nn.LayerNorm`` that may absorb the activation that follows it (fused HIP kernel)."""

    def __init__(self, *args, act: str = "none", **kwargs) -> None:
        super().__init__(*args, **kwargs)
        self.act = act

    def forward(self, x: Tensor) -> Tensor:
        if len(self.normalized_shape) != 1:
            return ops.reference.act_fn(super().forward(x), self.act)
        return ops.ln_act(x, self.weight, self.bias, self.eps, self.act)


class LayerNormChannelLast(nn.LayerNorm):
    """LayerNorm over the channel dim of an NCHW tensor (reference ``utils/model.py:225-235``).
    The fused kernel normalises in NCHW directly: no NHWC permute copies."""

    def __init__(self, *args, act: str = "none", **kwargs) -> None:
        super().__init__(*args, **kwargs)
        self.act = act

    def forward(self, x: Tensor) -> Tensor:
        if x.dim() != 4:
            raise ValueError(f"Input tensor must be 4D (NCHW), received {len(x.shape)}D instead: {x.shape}")
        if x.is_cuda and x.shape[0] * x.shape[2] * x.shape[3] < 8192:
            # few pixels (the env-interaction player): the per-pixel NCHW kernel is latency-bound
            # there, one wave per pixel row over channels-last data is not
            y = ops.ln_act(x.permute(0, 2, 3, 1).contiguous(), self.weight, self.bias, self.eps, self.act)
            return y.permute(0, 3, 1, 2)
        if x.is_contiguous(memory_format=torch.channels_last) and not x.is_contiguous():
            # NHWC storage (MIOpen's native conv layout): C is the innermost dim, a plain row LN
            y = ops.ln_act(x.permute(0, 2, 3, 1), self.weight, self.bias, self.eps, self.act)
            return y.permute(0, 3, 1, 2)
        return ops.ln_act_nchw(x, self.weight, self.bias, self.eps, self.act)


def fuse_norm_act(module: nn.Module) -> nn.Module:
    """In every ``nn.Sequential``: ``[nn.LayerNorm|LayerNormChannelLast, Act]`` -> fused norm + ``Identity``.
    Parameter names (``model.<i>.weight``) are preserved, so checkpoints keep their layout."""
    for child in module.modules():
        if not isinstance(child, nn.Sequential):
            continue
        mods = list(child._modules.items())
        for (name, m), (next_name, nxt) in zip(mods[:-1], mods[1:]):
            act = _ACT_NAMES.get(type(nxt))
            if act is None:
                continue
            if isinstance(m, (LayerNorm, LayerNormChannelLast)) and m.act == "none":
                m.act = act
                child._modules[next_name] = nn.Identity()
            elif type(m) is nn.LayerNorm and len(m.normalized_shape) == 1:
                fused = LayerNorm(m.normalized_shape, eps=m.eps, elementwise_affine=m.elementwise_affine,
                                  bias=m.bias is not None, act=act)
                fused.load_state_dict(m.state_dict())
                fused.to(device=m.weight.device if m.weight is not None else None)
                child._modules[name] = fused
                child._modules[next_name] = nn.Identity()
    return module
