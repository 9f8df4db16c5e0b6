"""Trial shards + loader (vspike.data, libvspike vs_shard_*): host-side input path, CPU only.
Byte work: the bar is exact equality with what was written."""
import os

import numpy as np
import pytest
import torch

from oracle import prng


@pytest.fixture(scope="module")
def shards(tmp_path_factory):
    from vspike import build
    from vspike.data import write_shard
    build.build(verbose=False)
    d = tmp_path_factory.mktemp("shards")
    out = []
    for s, (eid, n) in enumerate((("ses0", 7), ("ses1", 5))):
        video = (prng.uniform(100 + s, n * 12 * 24 * 20, "v") * 256).astype(np.uint8).reshape(n, 12, 1, 24, 20)
        ap = prng.spike_targets(200 + s, (n, 100, 9))
        keys = [f"{eid}_{t}" for t in range(n)]
        p = str(d / f"{eid}.vss")
        write_shard(p, video, ap, keys)
        out.append((p, video, ap, keys))
    return out


def test_shard_roundtrip_and_random_gather(shards):
    from vspike.data import TrialShard
    p, video, ap, keys = shards[0]
    sh = TrialShard(p)
    assert len(sh) == 7 and sh.video_shape == (12, 1, 24, 20) and sh.ap_shape == (100, 9)
    assert [sh.key(i) for i in range(7)] == keys
    idx = [6, 0, 3, 3, 1]
    v = torch.empty((5, 12, 1, 24, 20), dtype=torch.uint8)
    a = torch.empty((5, 100, 9), dtype=torch.float32)
    for threads in (1, 4):
        v.zero_(); a.zero_()
        sh.read(idx, v, a, threads=threads)
        assert np.array_equal(v.numpy(), video[idx]) and np.array_equal(a.numpy(), ap[idx])
    with pytest.raises(OSError):
        sh.read([7], v, a)
    with pytest.raises(IndexError):
        sh.key(7)
    rec = 4096 * (-(-12 * 24 * 20 // 4096)) + 4096 * (-(-100 * 9 * 4 // 4096))   # 4 KiB-aligned halves
    assert os.path.getsize(p) == 4096 + 7 * rec + 7 * 64


def test_shard_rejects_foreign_and_truncated_files(tmp_path, shards):
    from vspike.data import TrialShard
    bad = tmp_path / "x.vss"
    bad.write_bytes(b"not a shard" * 100)
    with pytest.raises(OSError):
        TrialShard(str(bad))
    p = shards[0][0]
    cut = tmp_path / "cut.vss"
    cut.write_bytes(open(p, "rb").read()[:8192])
    with pytest.raises(OSError):
        TrialShard(str(cut))


def test_loader_epoch_covers_every_trial_once(shards):
    from vspike.data import ShardLoader
    paths = [s[0] for s in shards]
    allv = np.concatenate([s[1] for s in shards])
    alla = np.concatenate([s[2] for s in shards])
    allk = sum((s[3] for s in shards), [])
    ld = ShardLoader(paths, batch_size=4, shuffle=True, seed=3, device="cpu", threads=3)
    assert len(ld) == 3
    seen = []
    for b in ld:
        assert set(b) == {"video", "ap", "eid", "__key__"}
        assert b["video"].dtype == torch.uint8 and b["ap"].dtype == torch.float32
        for j, k in enumerate(b["__key__"]):
            g = allk.index(k)
            assert np.array_equal(b["video"][j].numpy(), allv[g]) and np.array_equal(b["ap"][j].numpy(), alla[g])
            assert b["eid"][j] == k.split("_")[0]                # src/loader/base.py:40
        seen += b["__key__"]
    assert sorted(seen) == sorted(allk)
    first = [b["__key__"] for b in ShardLoader(paths, 4, seed=3, device="cpu")]
    again = [b["__key__"] for b in ShardLoader(paths, 4, seed=3, device="cpu")]
    assert first == again                                          # seeded order
    ld2 = ShardLoader(paths, 4, seed=3, device="cpu", drop_last=True)
    assert len(ld2) == 3 and all(len(b["__key__"]) == 4 for b in ld2)


@pytest.mark.parametrize("world", [2, 8])
@pytest.mark.parametrize("drop_last", [False, True])
def test_loader_data_parallel_ranks_split_each_global_batch(shards, tmp_path, world, drop_last):
    """every rank walks the same seeded permutation; each global batch
    (batch_size * world records) is cut into `world` disjoint per-rank slices."""
    from vspike.data import ShardLoader, write_shard
    n = 45                                                     # not a multiple of 2*3 nor 8*3
    video = (prng.uniform(300, n * 4 * 1 * 8 * 8, "v") * 256).astype(np.uint8).reshape(n, 4, 1, 8, 8)
    p = str(tmp_path / "dp.vss")
    write_shard(p, video, prng.spike_targets(301, (n, 100, 3)), [f"e{i % 3}_{i}" for i in range(n)])
    bs = 3
    loaders = [ShardLoader([p], bs, seed=5, device="cpu", rank=r, world=world, drop_last=drop_last)
               for r in range(world)]
    for epoch in range(2):
        per_rank = [[b["__key__"] for b in ld] for ld in loaders]
        nb = len(per_rank[0])
        assert all(len(x) == nb == len(loaders[0]) for x in per_rank)          # equal step counts
        assert all(len(k) == bs for x in per_rank for k in x)                   # full per-rank batches
        for step in range(nb):
            glob = [k for r in range(world) for k in per_rank[r][step]]
            if not (not drop_last and step == nb - 1):
                assert len(set(glob)) == bs * world                            # disjoint slices
        covered = {k for x in per_rank for b in x for k in b}
        if drop_last:
            assert nb == n // (bs * world) and len(covered) == nb * bs * world
        else:
            assert covered == {f"e{i % 3}_{i}" for i in range(n)}              # every record seen
        # identical permutation on every rank: the concatenated slices are one seeded order
        want = ShardLoader([p], bs * world, seed=5, device="cpu", drop_last=drop_last).rank_batches(epoch)
        for step in range(min(nb, len(want))):
            if len(want[step]) == bs * world:
                got = np.concatenate([loaders[r].rank_batches(epoch)[step] for r in range(world)])
                assert np.array_equal(got, want[step])
    with pytest.raises(ValueError):
        ShardLoader([p], bs, device="cpu", rank=world, world=world)
