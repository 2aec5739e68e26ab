"""Vectorised environments with gymnasium-0.29 autoreset semantics.

On ``terminated or truncated`` the sub-env is reset immediately; the returned observation is
the reset one and ``infos["final_observation"][i]`` / ``infos["final_info"][i]`` carry the
last step (with ``infos["_final_observation"]`` masks).  ``AsyncVectorEnv`` runs one worker
process per env (spawned, thunks shipped with cloudpickle) so emulator steps overlap with the
learner - the reference's ``gym.vector.AsyncVectorEnv`` role.
"""
from __future__ import annotations

import multiprocessing as mp
import sys
import traceback
from collections import OrderedDict
from typing import Any, Callable, Dict, List, Optional, Sequence, Union

import numpy as np

from sheeprl_prey_amd.envs import spaces


def _stack_obs(obs_list: List[Any], space: spaces.Space):
    if isinstance(space, spaces.Dict):
        return OrderedDict((k, np.stack([np.asarray(o[k]) for o in obs_list])) for k in space.keys())
    return np.stack([np.asarray(o) for o in obs_list])


def _add_info(infos: Dict[str, Any], info: Dict[str, Any], i: int, n: int) -> Dict[str, Any]:
    """gymnasium-0.29 layout: one array per key (numbers -> typed arrays, anything else - dicts
    included - -> object arrays with None) plus a ``_key`` presence mask."""
    for k, v in info.items():
        if k not in infos:
            if isinstance(v, (bool, np.bool_)):
                infos[k] = np.zeros(n, dtype=bool)
            elif isinstance(v, (int, np.integer)) and not isinstance(v, bool):
                infos[k] = np.zeros(n, dtype=np.int64)
            elif isinstance(v, (float, np.floating)):
                infos[k] = np.zeros(n, dtype=np.float64)
            else:
                infos[k] = np.full(n, None, dtype=object)
            infos[f"_{k}"] = np.zeros(n, dtype=bool)
        arr = infos[k]
        if arr.dtype != object and not isinstance(v, (bool, int, float, np.number, np.bool_)):
            obj = np.full(n, None, dtype=object)
            obj[:] = list(arr)
            infos[k] = arr = obj
        arr[i] = v
        infos[f"_{k}"][i] = True
    return infos


class VectorEnv:
    num_envs: int
    single_observation_space: spaces.Space
    single_action_space: spaces.Space
    observation_space: spaces.Space
    action_space: spaces.Space

    def _setup_spaces(self, obs_space, act_space):
        self.single_observation_space = obs_space
        self.single_action_space = act_space
        self.observation_space = spaces.batch_space(obs_space, self.num_envs)
        self.action_space = spaces.batch_space(act_space, self.num_envs)

    def _seeds(self, seed):
        if seed is None:
            return [None] * self.num_envs
        if isinstance(seed, int):
            return [seed + i for i in range(self.num_envs)]
        return list(seed)

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
        return False


class SyncVectorEnv(VectorEnv):
    def __init__(self, env_fns: Sequence[Callable[[], Any]], copy: bool = True):
        self.envs = [fn() for fn in env_fns]
        self.num_envs = len(self.envs)
        self._setup_spaces(self.envs[0].observation_space, self.envs[0].action_space)
        self.metadata = getattr(self.envs[0], "metadata", {})

    def reset(self, *, seed=None, options=None):
        obs, infos = [], {}
        for i, (env, s) in enumerate(zip(self.envs, self._seeds(seed))):
            o, info = env.reset(seed=s, options=options)
            obs.append(o)
            infos = _add_info(infos, info, i, self.num_envs)
        return _stack_obs(obs, self.single_observation_space), infos

    def step(self, actions):
        obs, rews, terms, truncs, infos = [], [], [], [], {}
        for i, env in enumerate(self.envs):
            a = actions[i]
            o, r, te, tr, info = env.step(a)
            if te or tr:
                old_o, old_info = o, info
                o, info = env.reset()
                info = dict(info)
                info["final_observation"] = old_o
                info["final_info"] = old_info
            obs.append(o)
            rews.append(r)
            terms.append(te)
            truncs.append(tr)
            infos = _add_info(infos, info, i, self.num_envs)
        return (
            _stack_obs(obs, self.single_observation_space),
            np.asarray(rews, dtype=np.float64),
            np.asarray(terms, dtype=bool),
            np.asarray(truncs, dtype=bool),
            infos,
        )

    def call(self, name: str, *args, **kwargs):
        out = []
        for env in self.envs:
            f = getattr(env, name)
            out.append(f(*args, **kwargs) if callable(f) else f)
        return tuple(out)

    def render(self):
        return self.envs[0].render()

    def close(self):
        for env in self.envs:
            env.close()


# ------------------------------------------------------------------ async
def _worker(remote, parent_remote, env_fn_bytes):
    import cloudpickle

    parent_remote.close()
    try:
        env = cloudpickle.loads(env_fn_bytes)()
    except Exception:  # pragma: no cover
        remote.send(("error", traceback.format_exc()))
        remote.close()
        return
    remote.send(("ok", (env.observation_space, env.action_space)))
    try:
        while True:
            cmd, data = remote.recv()
            if cmd == "reset":
                remote.send(("ok", env.reset(**data)))
            elif cmd == "step":
                o, r, te, tr, info = env.step(data)
                if te or tr:
                    old_o, old_info = o, info
                    o, info = env.reset()
                    info = dict(info)
                    info["final_observation"] = old_o
                    info["final_info"] = old_info
                remote.send(("ok", (o, r, te, tr, info)))
            elif cmd == "call":
                name, args, kwargs = data
                f = getattr(env, name)
                remote.send(("ok", f(*args, **kwargs) if callable(f) else f))
            elif cmd == "close":
                env.close()
                remote.send(("ok", None))
                break
    except (KeyboardInterrupt, EOFError):
        pass
    except Exception:  # pragma: no cover
        remote.send(("error", traceback.format_exc()))
    finally:
        remote.close()


class AsyncVectorEnv(VectorEnv):
    def __init__(self, env_fns: Sequence[Callable[[], Any]], context: Optional[str] = "spawn", daemon: bool = True):
        import cloudpickle

        self.num_envs = len(env_fns)
        # like gymnasium: build one env in the parent for the spaces (also lets make_env fill cfg keys)
        dummy = env_fns[0]()
        obs_space, act_space = dummy.observation_space, dummy.action_space
        self.metadata = getattr(dummy, "metadata", {})
        dummy.close()
        del dummy
        ctx = mp.get_context(context)
        self.remotes, self.processes = [], []
        for fn in env_fns:
            parent, child = ctx.Pipe()
            p = ctx.Process(target=_worker, args=(child, parent, cloudpickle.dumps(fn)), daemon=daemon)
            p.start()
            child.close()
            self.remotes.append(parent)
            self.processes.append(p)
        for r in self.remotes:
            status, payload = r.recv()
            if status != "ok":
                self.close(terminate=True)
                raise RuntimeError(f"env worker failed to start:\n{payload}")
        self._setup_spaces(obs_space, act_space)
        self.closed = False

    def _gather(self):
        out = []
        for r in self.remotes:
            status, payload = r.recv()
            if status != "ok":
                raise RuntimeError(f"env worker error:\n{payload}")
            out.append(payload)
        return out

    def reset(self, *, seed=None, options=None):
        for r, s in zip(self.remotes, self._seeds(seed)):
            r.send(("reset", {"seed": s, "options": options}))
        results = self._gather()
        infos: Dict[str, Any] = {}
        for i, (_, info) in enumerate(results):
            infos = _add_info(infos, info, i, self.num_envs)
        return _stack_obs([o for o, _ in results], self.single_observation_space), infos

    def step_async(self, actions) -> None:
        for r, a in zip(self.remotes, actions):
            r.send(("step", a))

    def step_wait(self):
        results = self._gather()
        infos: Dict[str, Any] = {}
        for i, res in enumerate(results):
            infos = _add_info(infos, res[4], i, self.num_envs)
        return (
            _stack_obs([res[0] for res in results], self.single_observation_space),
            np.asarray([res[1] for res in results], dtype=np.float64),
            np.asarray([res[2] for res in results], dtype=bool),
            np.asarray([res[3] for res in results], dtype=bool),
            infos,
        )

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def call(self, name: str, *args, **kwargs):
        for r in self.remotes:
            r.send(("call", (name, args, kwargs)))
        return tuple(self._gather())

    def close(self, terminate: bool = False):
        if getattr(self, "closed", False):
            return
        for r in self.remotes:
            try:
                r.send(("close", None))
            except (BrokenPipeError, EOFError, OSError):
                pass
        for r in self.remotes:
            try:
                r.recv()
            except (EOFError, OSError):
                pass
        for p in self.processes:
            p.join(timeout=5)
            if p.is_alive():
                p.terminate()
        self.closed = True

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
