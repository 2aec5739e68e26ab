"""sheeprl_prey_amd: an MI355X-native distributed RL framework with SheepRL's capabilities.

Importing the package registers every algorithm (reference ``sheeprl/__init__.py:14-25``)."""
import os

ROOT_DIR = os.path.dirname(os.path.abspath(__file__))
__version__ = "0.1.0"


def _register_algorithms() -> None:
    import importlib

    for mod in (
        "ppo.ppo",
        "ppo.ppo_decoupled",
        "ppo_recurrent.ppo_recurrent",
        "sac.sac",
        "sac.sac_decoupled",
        "sac_ae.sac_ae",
        "droq.droq",
        "dreamer_v1.dreamer_v1",
        "dreamer_v2.dreamer_v2",
        "dreamer_v3.dreamer_v3",
        "p2e_dv1.p2e_dv1",
        "p2e_dv2.p2e_dv2",
    ):
        try:
            importlib.import_module(f"sheeprl_prey_amd.algos.{mod}")
        except ModuleNotFoundError as e:
            if f"sheeprl_prey_amd.algos.{mod.split('.')[0]}" not in str(e):
                raise


_register_algorithms()
