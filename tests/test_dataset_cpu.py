"""Dataset codecs against the reference's own outputs (tests/golden/dataset.npz).

``Dataset.mirror`` (dataset.py:86-112) and ``Dataset.type_switch``
(dataset.py:114-171) are host-side table lookups here; they must reproduce
the reference loops element for element on the reference's self-play samples.
"""
import numpy as np

from match3tile.boardConfig import BoardConfig
from match3tile.dataset import Dataset, mirror_permutation


def _samples(g):
    k = len(g["task_seed"])
    obs = np.concatenate([g[f"task{i}_obs"] for i in range(k)])
    pol = np.concatenate([g[f"task{i}_pol"] for i in range(k)])
    val = np.concatenate([g[f"task{i}_val"] for i in range(k)])
    return obs, pol, val


def test_mirror_matches_reference(golden):
    g = golden("dataset")
    obs, pol, val = _samples(g)
    ds = Dataset(BoardConfig(seed=1)).with_mirroring(True)
    m = ds.mirror({"observations": list(obs), "policies": list(pol), "values": list(val)})
    assert np.array_equal(np.array(m["observations"]), g["mirror_obs"])
    assert np.array_equal(np.array(m["policies"]), g["mirror_pol"])
    assert np.array_equal(np.array(m["values"]), g["mirror_val"])


def test_mirror_permutation_is_an_involution():
    for shape in ((9, 9, 6), (16, 16, 8)):
        cfg = BoardConfig(seed=1, rows=shape[0], columns=shape[1], types=shape[2])
        perm = mirror_permutation(cfg)
        assert sorted(perm) == list(range(cfg.action_space))
        assert (perm[perm] == np.arange(cfg.action_space)).all()


def test_type_switch_matches_reference(golden):
    g = golden("dataset")
    obs, pol, val = _samples(g)
    ds = Dataset(BoardConfig(seed=1)).with_type_switching(True, 4)
    ds.dataset = {"observations": list(obs[:6]), "policies": list(pol[:6]), "values": list(val[:6])}
    ds._size = 6
    ds.type_switch()
    got = np.array([np.array(d["observations"]) for d in ds._type_switched_dataset])
    assert np.array_equal(got, g["switch_obs"])
    assert all(len(d["policies"]) == 3 for d in ds._type_switched_dataset)


def test_get_split_shapes_and_batches():
    ds = Dataset(BoardConfig(seed=1)).with_mirroring(True).with_batching(7)
    rng = np.random.default_rng(0)
    n = 40
    ds.dataset = {"observations": list(rng.integers(1, 7, (n, 9, 9))), "policies": list(rng.random((n, 144))),
                  "values": list(rng.integers(0, 500, n))}
    ds._size = n
    np.random.seed(3)
    train, test = ds.get_split(0.75)
    assert sum(len(b["values"]) for b in train) == 60 and sum(len(b["values"]) for b in test) == 20
    assert all(len(b["observations"]) <= 7 for b in train + test)
    assert max(b["values"].max() for b in train + test) <= 1.0
