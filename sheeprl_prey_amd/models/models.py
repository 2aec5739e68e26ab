"""Model building blocks (reference: ``sheeprl/models/models.py:15-489``).

Same constructor signatures and ``state_dict`` layout as the reference blocks; the forward
passes route through fused HIP ops (LayerNorm+act, LayerNorm-GRU epilogue) on GPU.
"""
from __future__ import annotations

import os
import warnings
from math import prod
from typing import Dict, Optional, Sequence, Union, no_type_check

import torch
import torch.nn.functional as F
from torch import Tensor, nn

from sheeprl_prey_amd import ops
from sheeprl_prey_amd.utils.model import ArgsType, ModuleType, cnn_forward, create_layers, fuse_norm_act, miniblock


class Linear(nn.Linear):
    """``nn.Linear`` (same parameters and state_dict) whose GPU backward takes the bias gradient with
    a parallel column-sum kernel (``ops.linear``)."""

    def forward(self, input: Tensor) -> Tensor:
        return ops.linear(input, self.weight, self.bias)


class MLP(nn.Module):
    """``[Linear -> dropout -> norm -> act] * len(hidden_sizes) (-> Linear(output_dim))``."""

    def __init__(
        self,
        input_dims: Union[int, Sequence[int]],
        output_dim: Optional[int] = None,
        hidden_sizes: Sequence[int] = (),
        layer_args: Optional[ArgsType] = None,
        dropout_layer: Optional[Union[ModuleType, Sequence[ModuleType]]] = None,
        dropout_args: Optional[ArgsType] = None,
        norm_layer: Optional[Union[ModuleType, Sequence[ModuleType]]] = None,
        norm_args: Optional[ArgsType] = None,
        activation: Optional[Union[ModuleType, Sequence[ModuleType]]] = nn.ReLU,
        act_args: Optional[ArgsType] = None,
        flatten_dim: Optional[int] = None,
    ) -> None:
        super().__init__()
        num_layers = len(hidden_sizes)
        if num_layers < 1 and output_dim is None:
            raise ValueError("The number of layers should be at least 1.")
        if isinstance(input_dims, Sequence) and flatten_dim is None:
            warnings.warn("input_dims is a sequence, but flatten_dim is not specified.")
        dropout_layer_list, dropout_args_list = create_layers(dropout_layer, dropout_args, num_layers)
        norm_layer_list, norm_args_list = create_layers(norm_layer, norm_args, num_layers)
        activation_list, act_args_list = create_layers(activation, act_args, num_layers)
        layer_args_list = layer_args if isinstance(layer_args, list) else [layer_args] * num_layers
        if isinstance(input_dims, int):
            input_dims = [input_dims]
        sizes = [prod(input_dims)] + list(hidden_sizes)
        model = []
        for i in range(num_layers):
            model += miniblock(
                sizes[i], sizes[i + 1], Linear, layer_args_list[i], dropout_layer_list[i], dropout_args_list[i],
                norm_layer_list[i], norm_args_list[i], activation_list[i], act_args_list[i],
            )
        if output_dim is not None:
            model += [Linear(sizes[-1], output_dim)]
        self._output_dim = output_dim or sizes[-1]
        self._model = fuse_norm_act(nn.Sequential(*model))
        self._flatten_dim = flatten_dim

    @property
    def model(self) -> nn.Module:
        return self._model

    @property
    def output_dim(self) -> int:
        return self._output_dim

    @property
    def flatten_dim(self) -> Optional[int]:
        return self._flatten_dim

    @no_type_check
    def forward(self, obs: Tensor) -> Tensor:
        if self.flatten_dim is not None:
            obs = obs.flatten(self.flatten_dim)
        return self.model(obs)


class _ConvStack(nn.Module):
    def __init__(
        self,
        input_channels: int,
        hidden_channels: Sequence[int],
        cnn_layer: ModuleType,
        layer_args: ArgsType = None,
        dropout_layer=None,
        dropout_args=None,
        norm_layer=None,
        norm_args=None,
        activation=nn.ReLU,
        act_args=None,
    ) -> None:
        super().__init__()
        num_layers = len(hidden_channels)
        if num_layers < 1:
            raise ValueError("The number of layers should be at least 1.")
        dropout_layer_list, dropout_args_list = create_layers(dropout_layer, dropout_args, num_layers)
        norm_layer_list, norm_args_list = create_layers(norm_layer, norm_args, num_layers)
        activation_list, act_args_list = create_layers(activation, act_args, num_layers)
        layer_args_list = layer_args if isinstance(layer_args, list) else [layer_args] * num_layers
        sizes = [input_channels] + list(hidden_channels)
        model = []
        for i in range(num_layers):
            model += miniblock(
                sizes[i], sizes[i + 1], cnn_layer, layer_args_list[i], dropout_layer_list[i], dropout_args_list[i],
                norm_layer_list[i], norm_args_list[i], activation_list[i], act_args_list[i],
            )
        self._output_dim = sizes[-1]
        self._model = fuse_norm_act(nn.Sequential(*model))

    @property
    def model(self) -> nn.Module:
        return self._model

    @property
    def output_dim(self) -> int:
        return self._output_dim

    def forward(self, obs: Tensor) -> Tensor:
        return self.model(obs)


class CNN(_ConvStack):
    """Conv2d stack (reference ``models.py:121-201``)."""

    def __init__(self, input_channels: int, hidden_channels: Sequence[int], cnn_layer: ModuleType = nn.Conv2d, **kwargs):
        super().__init__(input_channels, hidden_channels, cnn_layer, **kwargs)


class _NativeConvTranspose2d(nn.ConvTranspose2d):
    """``nn.ConvTranspose2d`` that never dispatches to MIOpen on the GPU.

    MIOpen's transposed-conv forward for the few-channel image output layer (measured: 8 -> 3,
    k4 s2 p1, N=64 at 32x32 -> 64x64) raised an illegal memory access on MI355X, depending on where
    its buffers sat in memory (reproduced under AMD_SERIALIZE_KERNEL=3: the fault is in MIOpen's own
    launch, profiles/r2_gpu_fault_note.md).  This layer runs PyTorch's native col2im transposed
    convolution instead; forward and backward are the same math, parameter names are unchanged.
    The DreamerV3 hot path does not use it: its decoder runs on the HIP conv stack (ops/conv.py)."""

    def forward(self, input: Tensor, output_size=None) -> Tensor:
        if input.is_cuda:
            with torch.backends.cudnn.flags(enabled=False):
                return super().forward(input, output_size)
        return super().forward(input, output_size)


class DeCNN(_ConvStack):
    """ConvTranspose2d stack (reference ``models.py:204-284``)."""

    def __init__(self, input_channels: int, hidden_channels: Sequence[int] = (), cnn_layer: ModuleType = nn.ConvTranspose2d,
                 **kwargs):
        super().__init__(input_channels, hidden_channels, cnn_layer, **kwargs)
        for m in self._model.modules():
            if type(m) is nn.ConvTranspose2d and m.out_channels <= 4:
                m.__class__ = _NativeConvTranspose2d


class NatureCNN(CNN):
    """DQN-Nature conv trunk 8s4/4s2/3s1 + fc + ReLU (reference ``models.py:287-327``)."""

    def __init__(self, in_channels: int, features_dim: int, screen_size: int = 64):
        super().__init__(
            in_channels,
            [32, 64, 64],
            layer_args=[{"kernel_size": 8, "stride": 4}, {"kernel_size": 4, "stride": 2}, {"kernel_size": 3, "stride": 1}],
        )
        with torch.no_grad():
            x = self.model(torch.rand(1, in_channels, screen_size, screen_size))
            out_dim = x.flatten(1).shape[1]
        self._output_dim = out_dim
        self.fc = None
        if features_dim is not None:
            self._output_dim = features_dim
            self.fc = nn.Linear(out_dim, features_dim)

    @property
    def output_dim(self) -> int:
        return self._output_dim

    def forward(self, x: Tensor) -> Tensor:
        if x.is_cuda and x.dtype == torch.float32 and ops.fused_enabled() and not self.training_eager:
            from sheeprl_prey_amd.ops.natcnn import conv_relu_plan, conv_relu_stack

            if not hasattr(self, "_nc_plan"):
                self._nc_plan = conv_relu_plan(self.model)
            if self._nc_plan is not None and x.shape[-3] == self._nc_plan[0].in_channels:
                # the three conv + ReLU layers on the implicit-GEMM HIP kernels (ops/natcnn.py)
                lead = x.shape[:-3]
                y = conv_relu_stack(self._nc_plan, x.reshape(-1, *x.shape[-3:]))
                x = y.reshape(*lead, -1)
                return F.relu(self.fc(x)) if self.fc is not None else x
        x = cnn_forward(self.model, x, input_dim=x.shape[-3:], output_dim=(-1,))
        return F.relu(self.fc(x)) if self.fc is not None else x

    training_eager = False  # True: the stock conv path (tests toggle it)


class LayerNormGRUCell(nn.Module):
    """GRU cell with LayerNorm on the input projection (reference ``models.py:330-402``).

    ``x = Linear([h, input])``; ``LN``; ``r = sig``, ``c = tanh(r*c)``, ``u = sig(u-1)``;
    ``h' = u*c + (1-u)*h``.  On GPU the LN+gates epilogue is ONE fused kernel (fwd and bwd)."""

    def __init__(self, input_size: int, hidden_size: int, bias: bool = True, batch_first: bool = False,
                 layer_norm: bool = False) -> None:
        super().__init__()
        self.input_size = input_size
        self.hidden_size = hidden_size
        self.bias = bias
        self.batch_first = batch_first
        self.linear = nn.Linear(input_size + hidden_size, 3 * hidden_size, bias=self.bias)
        self.layer_norm = nn.LayerNorm(3 * hidden_size) if layer_norm else nn.Identity()

    def project(self, input: Tensor, hx: Tensor) -> Tensor:
        return self.linear(torch.cat((hx, input), -1))

    def gates(self, x: Tensor, hx: Tensor) -> Tensor:
        if isinstance(self.layer_norm, nn.LayerNorm):
            return ops.ln_gru(x, hx, self.layer_norm.weight, self.layer_norm.bias, self.layer_norm.eps)
        reset, cand, update = torch.chunk(x, 3, -1)
        reset = torch.sigmoid(reset)
        cand = torch.tanh(reset * cand)
        update = torch.sigmoid(update - 1)
        return update * cand + (1 - update) * hx

    def forward(self, input: Tensor, hx: Optional[Tensor] = None) -> Tensor:
        is_3d = input.dim() == 3
        if is_3d:
            if input.shape[int(self.batch_first)] == 1:
                input = input.squeeze(int(self.batch_first))
            else:
                raise AssertionError(
                    "LayerNormGRUCell: Expected input to be 3-D with sequence length equal to 1 but received "
                    f"a sequence of length {input.shape[int(self.batch_first)]}"
                )
        if hx is not None and hx.dim() == 3:
            hx = hx.squeeze(0)
        assert input.dim() in (1, 2), f"LayerNormGRUCell: Expected input to be 1-D or 2-D but received {input.dim()}-D tensor"
        is_batched = input.dim() == 2
        if not is_batched:
            input = input.unsqueeze(0)
        if hx is None:
            hx = torch.zeros(input.size(0), self.hidden_size, dtype=input.dtype, device=input.device)
        else:
            hx = hx.unsqueeze(0) if not is_batched else hx
        hx = self.gates(self.project(input, hx), hx)
        if not is_batched:
            hx = hx.squeeze(0)
        elif is_3d:
            hx = hx.unsqueeze(0)
        return hx


class MultiEncoder(nn.Module):
    """Concatenate CNN and MLP features (reference ``models.py:405-460``)."""

    def __init__(self, cnn_encoder: Optional[nn.Module], mlp_encoder: Optional[nn.Module]) -> None:
        super().__init__()
        if cnn_encoder is None and mlp_encoder is None:
            raise ValueError("There must be at least one encoder, both cnn and mlp encoders are None")
        self.has_cnn_encoder = cnn_encoder is not None
        self.has_mlp_encoder = mlp_encoder is not None
        if self.has_cnn_encoder and getattr(cnn_encoder, "input_dim", None) is None:
            raise AttributeError("`cnn_encoder` must contain the `input_dim` attribute")
        if self.has_cnn_encoder and getattr(cnn_encoder, "output_dim", None) is None:
            raise AttributeError("`cnn_encoder` must contain the `output_dim` attribute")
        if self.has_mlp_encoder and getattr(mlp_encoder, "input_dim", None) is None:
            raise AttributeError("`mlp_encoder` must contain the `input_dim` attribute")
        if self.has_mlp_encoder and getattr(mlp_encoder, "output_dim", None) is None:
            raise AttributeError("`mlp_encoder` must contain the `output_dim` attribute")
        self.cnn_encoder = cnn_encoder
        self.mlp_encoder = mlp_encoder
        self.cnn_output_dim = cnn_encoder.output_dim if cnn_encoder is not None else 0
        self.mlp_output_dim = mlp_encoder.output_dim if mlp_encoder is not None else 0
        self.output_dim = self.cnn_output_dim + self.mlp_output_dim

    def forward(self, obs: Dict[str, Tensor], *args, **kwargs) -> Tensor:
        if self.has_cnn_encoder:
            cnn_out = self.cnn_encoder(obs, *args, **kwargs)
        if self.has_mlp_encoder:
            mlp_out = self.mlp_encoder(obs, *args, **kwargs)
        if self.has_cnn_encoder and self.has_mlp_encoder:
            return torch.cat((cnn_out, mlp_out), -1)
        return cnn_out if self.has_cnn_encoder else mlp_out


class MultiDecoder(nn.Module):
    """Merge the dicts of reconstructions of a CNN and an MLP decoder (reference ``models.py:463-489``)."""

    def __init__(self, cnn_decoder: Optional[nn.Module], mlp_decoder: Optional[nn.Module]) -> None:
        super().__init__()
        if cnn_decoder is None and mlp_decoder is None:
            raise ValueError("There must be an decoder, both cnn and mlp decoders are None")
        self.cnn_decoder = cnn_decoder
        self.mlp_decoder = mlp_decoder

    def forward(self, x: Tensor, onehot=None) -> Dict[str, Tensor]:
        """``onehot`` (optional ``(idx, G, off, n_onehot)``): the first ``n_onehot`` latent columns are
        one-hot (DreamerV3 posteriors); decoders that support it gather them (``ops/onehot.py``)."""
        reconstructed_obs = {}
        kw = {"onehot": onehot} if onehot is not None else {}
        if self.cnn_decoder is not None:
            reconstructed_obs.update(self.cnn_decoder(x, **kw))
        if self.mlp_decoder is not None:
            reconstructed_obs.update(self.mlp_decoder(x, **kw))
        return reconstructed_obs
