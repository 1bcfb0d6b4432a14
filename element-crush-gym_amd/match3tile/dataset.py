"""Self-play dataset producer and codecs over the device MCTS.

Drop-in for the reference's ``dataset.py``:

* ``mcts_task(data)`` -- dataset.py:16-43: MCTS(state, 3, 256) self-play
  games until more than ``batch_size`` samples, each move recording
  ``(observation int64 [R, C], policy float [A], value)``; the value of every
  sample is the game's final reward. The policy vector keeps the reference's
  pairing of ``state.legal_actions`` (ascending) with the root's child visit
  shares (expansion order) verbatim.
* ``Dataset`` -- dataset.py:46-260: ``sample`` (pickle cache file
  ``"(R, C, T).ds"`` holding the same dict of lists), ``mirror`` (left-right
  flip of boards and the matching action permutation), ``type_switch`` (token
  relabelling over permutations), ``get_split`` / batching.
* ``play_games`` -- the batched producer: many games in lockstep, every MCTS
  simulation of every game sharing ONE rollout launch; game g with its own
  ``random.Random(pyseeds[g])`` produces exactly what ``mcts_task`` produces
  after ``random.seed(pyseeds[g])``.

The mirror and type-switch codecs are table lookups (numpy), equal element
for element to the reference loops.
"""
from __future__ import annotations

import math
import os
import pickle
import random
from itertools import permutations
from typing import Sequence

import numpy as np

from .boardConfig import BoardConfig
from .boardv2 import BoardV2
from .mcts import MCTS, search_lockstep

SIMULATIONS = 256        # dataset.py:29
EXPLORATION = 3


def _policy_vector(cfg, legal, shares):
    pol = np.zeros(cfg.action_space)
    for a, p in zip(legal, shares):                 # dataset.py:32-34 (pairs by position)
        pol[a] = p
    return pol


def mcts_task(data):
    """dataset.py:16-43 on the device MCTS: ((callback, (cfg, moves)), batch_size) -> [samples]."""
    (callback, (cfg, moves)), batch_size = data
    out = {"observations": [], "policies": [], "values": []}
    count = 0
    while count <= batch_size:
        state = BoardV2(moves, cfg)
        search = MCTS(state, EXPLORATION, SIMULATIONS, False, False)
        while not state.is_terminal:
            action, _, shares = search()
            out["observations"].append(state.array)
            out["policies"].append(_policy_vector(state.cfg, state.legal_actions, shares))
            state = state.apply_action(action)
            count += 1
            callback()
        out["values"].extend([state.reward] * moves)
    return [out]


def play_games(cfgs: Sequence[BoardConfig], moves: int, pyseeds: Sequence[int], simulations: int = SIMULATIONS,
               exploration_weight: float = EXPLORATION, leaf_rollouts: int = 1, rollout_fn=None):
    """One self-play game per cfg, all in lockstep (one rollout launch per simulation round).

    Returns the same dict of lists as ``mcts_task``, games in order."""
    games = []
    for cfg, ps in zip(cfgs, pyseeds):
        rng = random.Random(ps)
        state = BoardV2(moves, cfg)
        games.append({"state": state, "rng": rng, "obs": [], "pol": [],
                      "mcts": MCTS(state, exploration_weight, simulations, False, False, leaf_rollouts,
                                   rollout_fn, rng)})
    live = [g for g in games if not g["state"].is_terminal]
    while live:
        results = search_lockstep([g["mcts"] for g in live])
        for g, (action, _, shares) in zip(live, results):
            st = g["state"]
            g["obs"].append(st.array)
            g["pol"].append(_policy_vector(st.cfg, st.legal_actions, shares))
            g["state"] = st.apply_action(action)
        live = [g for g in live if not g["state"].is_terminal]
    out = {"observations": [], "policies": [], "values": []}
    for g in games:
        out["observations"].extend(g["obs"])
        out["policies"].extend(g["pol"])
        out["values"].extend([g["state"].reward] * moves)
    return out


def mirror_permutation(cfg) -> np.ndarray:
    """perm[a] = id of action a on the left-right mirrored board (dataset.py:95-103)."""
    perm = np.empty(cfg.action_space, dtype=np.int64)
    for a in range(cfg.action_space):
        (r1, c1), (r2, c2) = cfg.decode(a)
        perm[a] = cfg.encode((r1, cfg.columns - 1 - c1), (r2, cfg.columns - 1 - c2))
    return perm


def type_switch_tables(cfg, limit: int) -> np.ndarray:
    """Row i-1 = token -> new value for the i-th permutation of 1..T+1 (dataset.py:128-150), i = 1..limit."""
    rows = []
    for i, perm in enumerate(permutations(range(1, cfg.types + 2))):
        if i == 0:
            continue
        if i == limit + 1:
            break
        lut = np.full(cfg.type_mask + 1, -1, dtype=np.int64)   # tokens without a letter have no mapping
        lut[0] = cfg.mega_token                                # 'x'
        lut[1:cfg.types + 2] = perm
        rows.append(lut)
    return np.array(rows, dtype=np.int64).reshape(-1, cfg.type_mask + 1)


class Dataset:
    """dataset.py:46-260 with the device self-play producer."""

    def __init__(self, cfg: BoardConfig, moves: int = 20):
        self.cfg = cfg
        self.moves = moves
        self._size = 0
        self._mirroring = False
        self._batching = 1
        self._type_switching = False
        self._type_switching_limit = -1
        self.dataset = {"observations": [], "policies": [], "values": []}
        self._type_switched_dataset: list = []

    @property
    def cache_file(self) -> str:
        return str((*self.cfg.shape, self.cfg.types)) + ".ds"

    def sample(self, size, caching=True, games_per_launch: int = 256):
        """Grow the dataset to `size` (rounded up to 20) samples; cached in ``cache_file`` (pickle)."""
        size = 20 * math.ceil(size / 20)
        if caching and os.path.isfile(self.cache_file) and not self.dataset["values"]:
            with open(self.cache_file, "rb") as f:  # a file this class wrote (same format as the reference)
                self.dataset = pickle.load(f)
        missing = size - len(self.dataset["values"])
        while missing > 0:
            # every game starts from self.cfg's board, as the reference's workers do
            # (dataset.py:72 hands the one cfg to every mcts_task); each game gets
            # its own Python RNG seed for the rollouts
            n = min(games_per_launch, max(1, math.ceil(missing / self.moves)))
            seeds = [random.randint(0, 2**31 - 1) for _ in range(n)]
            batch = play_games([self.cfg] * n, self.moves, seeds)
            for k, v in batch.items():
                self.dataset[k].extend(v)
            missing = size - len(self.dataset["values"])
        if caching:
            with open(self.cache_file, "wb") as f:
                pickle.dump(self.dataset, f)
        self._size = size
        return self

    def mirror(self, data):
        if not self._mirroring:
            return data
        perm = mirror_permutation(self.cfg)
        n = len(data["values"])
        obs = np.asarray(data["observations"][:n])
        pol = np.asarray(data["policies"][:n], dtype=np.float64)
        flipped = obs[:, :, ::-1]
        mpol = np.zeros_like(pol)
        mpol[:, perm] = pol
        data["observations"].extend(list(flipped))
        data["policies"].extend(list(mpol))
        data["values"].extend(list(data["values"][:n]))
        return data

    def switch_observations(self, obs: np.ndarray, lower: int, limit: int) -> list:
        """The `switch` closure of dataset.py:128-155: permutations lower..limit of one board."""
        if lower >= limit:
            return []
        tabs = type_switch_tables(self.cfg, limit)
        tokens = obs & self.cfg.type_mask
        special = obs & self.cfg.special_type_mask
        out = []
        for i in range(max(lower, 1), limit + 1):
            new = tabs[i - 1][tokens]
            if (new < 0).any():
                raise TypeError("token without a type letter (reference: None in np.vectorize)")
            out.append(new + special)
        return out

    def type_switch(self):
        if not self._type_switching:
            return
        limit = self._type_switching_limit
        if limit <= 0:
            limit = math.factorial(self.cfg.types)
        limit -= 1
        for i, obs in enumerate(self.dataset["observations"][:self._size]):
            obs = np.asarray(obs)
            if i < len(self._type_switched_dataset):
                have = len(self._type_switched_dataset[i]["observations"])
                if have >= limit:
                    continue
                d = self._type_switched_dataset[i]
                d["observations"].extend(self.switch_observations(obs, have, limit))
                d["policies"].extend(self.dataset["policies"][i] * (limit - have))
                d["values"].extend(self.dataset["values"][i] * (limit - have))
            else:
                self._type_switched_dataset.append({
                    "observations": self.switch_observations(obs, 1, limit),
                    "policies": [self.dataset["policies"][i]] * limit,
                    "values": [self.dataset["values"][i]] * limit,
                })

    def with_mirroring(self, should_mirror):
        self._mirroring = should_mirror
        return self

    def with_batching(self, batch_size):
        self._batching = batch_size
        return self

    def with_type_switching(self, should_switch, switch_limit):
        self._type_switching = should_switch
        self._type_switching_limit = min(switch_limit, math.factorial(self.cfg.types + 1))
        return self

    def get_split(self, split=0.8):
        data = {k: list(v[:self._size]) for k, v in self.dataset.items()}
        self.type_switch()
        for sw in self._type_switched_dataset:
            for k, v in sw.items():
                data[k].extend(v[:self._size])
        data = self.mirror(data)
        if not (0 < split < 1):
            raise ValueError("Split value must be between 0 and 1.")
        obs = np.array(data["observations"])
        pol = np.array(data["policies"])
        val = np.array(data["values"]) / np.max(self.dataset["values"])
        if not (len(obs) == len(pol) == len(val)):
            raise ValueError("All input data arrays must have the same length.")
        idx = np.arange(len(obs))
        np.random.shuffle(idx)                        # numpy's global RNG, as the reference
        obs, pol, val = obs[idx], pol[idx], val[idx]
        cut = int(len(obs) * split)

        def batches(o, p, v):
            nb = math.ceil(len(o) / self._batching)
            return [{"observations": o[i * self._batching:(i + 1) * self._batching],
                     "policies": p[i * self._batching:(i + 1) * self._batching],
                     "values": v[i * self._batching:(i + 1) * self._batching]} for i in range(nb)]

        return batches(obs[:cut], pol[:cut], val[:cut]), batches(obs[cut:], pol[cut:], val[cut:])
