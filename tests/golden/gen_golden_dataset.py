#!/usr/bin/env python3
"""Golden vectors for the dataset producer/codec, from the REAL reference.

    PYTHONPATH=/root/reference python3 -B tests/golden/gen_golden_dataset.py

Runs in this container only. Writes ``tests/golden/dataset.npz``:

  task_*     ``dataset.mcts_task`` (dataset.py:16-43) -- MCTS(state, 3, 256)
             self-play, one game of 5 moves per (cfg seed, Python random seed):
             observations int64 [k][9][9], policies float [k][144], values;
  mirror_*   ``Dataset.mirror`` (dataset.py:86-112) of those samples;
  switch_*   ``Dataset.type_switch`` (dataset.py:114-171) with limit 4 on the
             first samples: the switched observations.

Only data is committed -- no reference source.
"""
from __future__ import annotations

import os
import random
import sys
from multiprocessing import Pool

sys.dont_write_bytecode = True
REF = os.environ.get("M3_REFERENCE", "/root/reference")
if REF not in sys.path:
    sys.path.insert(0, REF)

import numpy as np  # noqa: E402

import dataset as ref_dataset  # noqa: E402
from match3tile.boardConfig import BoardConfig  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
MOVES = 5
CASES = [(7, 101), (19, 202), (33, 303)]  # (cfg seed, Python random seed)


def _task(args):
    seed, pyseed = args
    cfg = BoardConfig(seed=seed)
    random.seed(pyseed)
    (data,) = ref_dataset.mcts_task(((lambda: None, (cfg, MOVES)), MOVES - 1))
    return (np.array(data["observations"], dtype=np.int64), np.array(data["policies"], dtype=np.float64),
            np.array(data["values"], dtype=np.int64))


def main():
    with Pool(len(CASES)) as pool:
        res = pool.map(_task, CASES)
    out = {"task_seed": np.array([c[0] for c in CASES]), "task_pyseed": np.array([c[1] for c in CASES]),
           "task_moves": np.array(MOVES)}
    for i, (obs, pol, val) in enumerate(res):
        out[f"task{i}_obs"], out[f"task{i}_pol"], out[f"task{i}_val"] = obs, pol, val
    obs = np.concatenate([r[0] for r in res])
    pol = np.concatenate([r[1] for r in res])
    val = np.concatenate([r[2] for r in res])
    ds = ref_dataset.Dataset(BoardConfig(seed=1)).with_mirroring(True)
    m = ds.mirror({"observations": list(obs), "policies": list(pol), "values": list(val)})
    out["mirror_obs"] = np.array(m["observations"], dtype=np.int64)
    out["mirror_pol"] = np.array(m["policies"], dtype=np.float64)
    out["mirror_val"] = np.array(m["values"], dtype=np.int64)
    # type switching of the first samples (boards with specials included)
    ds2 = ref_dataset.Dataset(BoardConfig(seed=1)).with_type_switching(True, 4)
    ds2.dataset = {"observations": list(obs[:6]), "policies": list(pol[:6]), "values": list(val[:6])}
    ds2._size = 6
    ds2.type_switch()
    out["switch_in"] = obs[:6]
    out["switch_obs"] = np.array([np.array(d["observations"]) for d in ds2._type_switched_dataset], dtype=np.int64)
    np.savez_compressed(os.path.join(OUT, "dataset.npz"), **out)
    print({k: getattr(v, "shape", v) for k, v in out.items()})


if __name__ == "__main__":
    main()
