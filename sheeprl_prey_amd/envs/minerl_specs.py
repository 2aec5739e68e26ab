"""Custom MineRL 0.4.4 tasks (reference ``sheeprl/envs/minerl_envs/{backend,navigate,obtain}.py``):
``custom_navigate`` (optionally dense/extreme) and ``custom_obtain_{diamond,iron_pickaxe}`` with a
block-breaking speed multiplier.  The task contents are data tables; the herobraine ``EnvSpec``
subclass is assembled on demand, so importing this module never needs MineRL."""
from __future__ import annotations

from typing import Any, Dict, List

from sheeprl_prey_amd.envs._gate import require

NAVIGATE_STEPS = 6000
SIMPLE_KEYS = ("forward", "back", "left", "right", "jump", "sneak", "sprint", "attack")
OBTAIN_INVENTORY = ["dirt", "coal", "torch", "log", "planks", "stick", "crafting_table", "wooden_axe",
                    "wooden_pickaxe", "stone", "cobblestone", "furnace", "stone_axe", "stone_pickaxe", "iron_ore",
                    "iron_ingot", "iron_axe", "iron_pickaxe"]
TOOLS = ["wooden_axe", "wooden_pickaxe", "stone_axe", "stone_pickaxe", "iron_axe", "iron_pickaxe"]
OBTAIN_ACTIONS = {
    "PlaceBlock": ["dirt", "stone", "cobblestone", "crafting_table", "furnace", "torch"],
    "EquipAction": ["air"] + TOOLS,
    "CraftAction": ["torch", "stick", "planks", "crafting_table"],
    "CraftNearbyAction": TOOLS + ["furnace"],
    "SmeltItemNearby": ["iron_ingot", "coal"],
}
_LADDER = [("log", 1), ("planks", 2), ("stick", 4), ("crafting_table", 4), ("wooden_pickaxe", 8),
           ("cobblestone", 16), ("furnace", 32), ("stone_pickaxe", 32), ("iron_ore", 64), ("iron_ingot", 128),
           ("iron_pickaxe", 256), ("diamond", 1024)]
OBTAIN_TASKS = {
    "diamond": dict(schedule=_LADDER, max_steps=18000, quit=("possess", "diamond")),
    "iron_pickaxe": dict(schedule=_LADDER[:-1], max_steps=6000, quit=("craft", "iron_pickaxe")),
}


def _camel(s: str) -> str:
    return "".join(w.capitalize() for w in s.split("_"))


def make_spec(id: str, break_speed: int = 100, dense: bool = False, extreme: bool = False, **kwargs: Any):
    """Build the herobraine env spec for ``id``; ``.make()`` on the result creates the gym env."""
    require("minerl", "Install minerl==0.4.4 to use `env=minerl`.")
    from minerl.herobraine.env_spec import EnvSpec
    from minerl.herobraine.hero import handler, handlers
    from minerl.herobraine.hero.mc import INVERSE_KEYMAP, MS_PER_STEP

    class BreakSpeed(handler.Handler):
        def __init__(self, multiplier: float):
            self.multiplier = multiplier

        def to_string(self):
            return f"break_speed({self.multiplier})"

        def xml_template(self):
            return "<BreakSpeedMultiplier>{{multiplier}}</BreakSpeedMultiplier>"

    task = id.lower()
    if task == "custom_navigate":
        name = "CustomMineRLNavigate{}{}-v0".format("Extreme" if extreme else "", "Dense" if dense else "")
        max_steps = NAVIGATE_STEPS
        extra_obs = [handlers.CompassObservation(angle=True, distance=False), handlers.FlatInventoryObservation(["dirt"])]
        extra_act = [handlers.PlaceBlock(["none", "dirt"], _other="none", _default="none")]
        rewards = [handlers.RewardForTouchingBlockType([{"type": "diamond_block", "behaviour": "onceOnly",
                                                          "reward": 100.0}])]
        if dense:
            rewards.append(handlers.RewardForDistanceTraveledToCompassTarget(reward_per_block=1.0))
        start = [handlers.SimpleInventoryAgentStart([dict(type="compass", quantity="1")])]
        agent = [handlers.AgentQuitFromTouchingBlockType(["diamond_block"])]
        worldgen = [handlers.BiomeGenerator(biome=3, force_reset=True) if extreme
                    else handlers.DefaultWorldGenerator(force_reset=True)]
        quits, initial = [], []
    elif task.startswith("custom_obtain_"):
        target = task[len("custom_obtain_"):]
        t = OBTAIN_TASKS[target]
        name = "CustomMineRLObtain{}{}-v0".format(_camel(target), "Dense" if dense else "")
        max_steps = t["max_steps"]
        extra_obs = [handlers.FlatInventoryObservation(OBTAIN_INVENTORY),
                     handlers.EquippedItemObservation(items=["air"] + TOOLS + ["other"], _default="air", _other="other")]
        extra_act = [getattr(handlers, h)(["none"] + items, _other="none", _default="none")
                     for h, items in OBTAIN_ACTIONS.items()]
        sched = [dict(type=k, amount=1, reward=r) for k, r in t["schedule"]]
        rewards = [(handlers.RewardForCollectingItems if dense else handlers.RewardForCollectingItemsOnce)(sched)]
        start = []
        kind, item = t["quit"]
        agent = [(handlers.AgentQuitFromPossessingItem if kind == "possess" else handlers.AgentQuitFromCraftingItem)(
            [dict(type=item, amount=1)])]
        worldgen = [handlers.DefaultWorldGenerator(force_reset=True)]
        quits = [handlers.ServerQuitFromTimeUp(time_limit_ms=max_steps * MS_PER_STEP),
                 handlers.ServerQuitWhenAnyAgentFinishes()]
        initial = [handlers.TimeInitialCondition(start_time=6000, allow_passage_of_time=True),
                   handlers.SpawningInitialCondition(allow_spawning=True)]
    else:
        raise ValueError(f"Unknown MineRL task `{id}`; expected custom_navigate / custom_obtain_diamond / "
                         "custom_obtain_iron_pickaxe")

    resolution = tuple(kwargs.pop("resolution", (64, 64)))

    class Spec(EnvSpec):
        def create_observables(self) -> List:
            return [handlers.POVObservation(resolution), handlers.ObservationFromCurrentLocation(),
                    handlers.ObservationFromLifeStats()] + extra_obs

        def create_actionables(self) -> List:
            return [handlers.KeybasedCommandAction(k, v) for k, v in INVERSE_KEYMAP.items() if k in SIMPLE_KEYS] + \
                [handlers.CameraAction()] + extra_act

        def create_rewardables(self):
            return rewards

        def create_agent_start(self):
            return [BreakSpeed(break_speed)] + start

        def create_agent_handlers(self):
            return agent

        def create_server_world_generators(self):
            return worldgen

        def create_server_quit_producers(self):
            return quits

        def create_server_decorators(self):
            return []

        def create_server_initial_conditions(self):
            return initial

        def create_monitors(self):
            return []

        def is_from_folder(self, folder: str) -> bool:
            return False

        def get_docstring(self) -> str:
            return name

        def determine_success_from_rewards(self, rewards_seen: list) -> bool:
            return False

    return Spec(name, max_episode_steps=max_steps)


def task_kwargs(id: str, kwargs: Dict[str, Any]) -> Dict[str, Any]:
    out = dict(kwargs)
    if "navigate" not in id.lower():
        out.pop("extreme", None)
    return out
