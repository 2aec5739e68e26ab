"""World-model container shared by the Dreamer family (reference ``dreamer_v2/agent.py:630-655``)."""
from typing import Optional

from torch import nn


class WorldModel(nn.Module):
    def __init__(self, encoder: nn.Module, rssm: nn.Module, observation_model: nn.Module, reward_model: nn.Module,
                 continue_model: Optional[nn.Module]) -> None:
        super().__init__()
        self.encoder = encoder
        self.rssm = rssm
        self.observation_model = observation_model
        self.reward_model = reward_model
        self.continue_model = continue_model
