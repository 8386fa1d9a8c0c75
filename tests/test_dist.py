"""Multi-rank path on CPU: static sharding, the stats all-gather (gloo, world size 2, the
same orchestration code the RCCL path runs), the unique-id bootstrap, and the dataset
metrics against a single-process computation (processing_utils/evaluate.py formula)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

from conftest import ROOT
from oracle import tic_oracle as o
from tf_image_compression_amd import dist, sharded


@pytest.mark.parametrize("n,world", [(10, 2), (10000, 8), (7, 8), (0, 3), (1250, 1)])
def test_shard_range_partitions(n, world):
    seen = []
    for r in range(world):
        lo, hi = dist.shard_range(n, r, world)
        assert 0 <= lo <= hi <= n
        seen.extend(range(lo, hi))
    assert seen == list(range(n))


def test_combine_matches_dataset_psnr():
    r = np.random.default_rng(0)
    a = [r.integers(0, 256, (8, 9, 3), dtype=np.uint8) for _ in range(5)]
    b = [np.clip(x.astype(int) + r.integers(-5, 6, x.shape), 0, 255).astype(np.uint8) for x in a]
    sts = []
    for k in range(5):
        s = dist.RankStats(sse=float(np.sum((a[k].astype(float) - b[k]) ** 2)), dims=a[k].size, bits=100,
                           images=1, t_start=k, t_end=k + 1)
        sts.append(dist.RankStats.from_array(s.to_array()))
    res = dist.combine(sts)
    assert abs(res["psnr_db"] - o.dataset_psnr(list(zip(a, b)))) < 1e-9
    assert res["images"] == 5 and abs(res["bpp"] - 500 / (5 * 72)) < 1e-12 and res["seconds"] == 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("driver", ["host", "device"])
def test_gloo_world2_sharded_stats(tmp_path, driver):
    """Both shard drivers over gloo at world size 2: "host" (run_shard) and "device"
    (run_device_shard, the GPU path's orchestration: resident shard, batches at buffer
    offsets, one SSE reduction, one all-gather) with tests/host_codec.py standing in for
    the GPU codec."""
    n, P = 7, 32
    port = _free_port()
    out = str(tmp_path / "res")
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS="2")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tests", "dist_worker.py"),
           out, str(n), str(P), driver]
    subprocess.run(cmd, check=True, env=env, timeout=240, cwd=ROOT)
    res = [json.load(open(f"{out}.{r}")) for r in range(2)]
    assert res[0]["summary"] == res[1]["summary"]
    assert res[0]["images"] == [4, 3] and all(x["uid_ok"] for x in res) and res[0]["tmax"] == 2.0
    assert res[0]["gather"] == res[1]["gather"] == [[0, 10, 7.5], [1, 11, 7.5]]
    # single-process reference over the whole set
    from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD
    params = synthetic_params(1)
    x = sharded.image_batch(0, n, P)
    _, idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, P, 2, 1)
    y = o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, 1)[1]
    psnr = o.dataset_psnr(list(zip(x, y)))
    assert abs(res[0]["summary"]["psnr_db"] - psnr) < 1e-6
    assert res[0]["summary"]["bpp"] == pytest.approx(0.25)


def test_unique_id_bytes_keep_zeros():
    """The 128-byte ncclUniqueId passes through the TCP bootstrap as raw bytes: zero bytes
    inside it (sockaddr padding) must survive extraction and re-packing (round 1 read it
    through a c_char field, which cuts at the first NUL)."""
    raw = bytes([0, 2, 0, 0, 127, 0, 0, 1] + [0] * 40 + list(range(80)))
    uid = dist.uid_from_bytes(raw)
    assert dist.uid_to_bytes(uid) == raw
    with pytest.raises(ValueError):
        dist.uid_from_bytes(raw[:-1])


def _uid_peer(rank, world, port, q):
    from tf_image_compression_amd.dist import exchange_unique_id
    payload = bytes([0, 7, 0, 0, 255] + list(range(123))) if rank == 0 else None
    q.put((rank, exchange_unique_id(rank, world, payload, "127.0.0.1", port, timeout=60.0)))


def test_unique_id_exchange_world3():
    """The ncclUniqueId bootstrap of RcclComm (dist.exchange_unique_id): rank 0 serves the
    128 bytes over TCP and every peer — started before or after the server — receives them
    intact, zero bytes included (the RCCL path of an N>1 bench run, without a GPU)."""
    import multiprocessing as mp
    import socket
    with socket.socket() as s:  # a free port on the loopback interface
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_uid_peer, args=(r, 3, port, q)) for r in (2, 1, 0)]  # peers first
    for p in procs:
        p.start()
    got = dict(q.get(timeout=90) for _ in procs)
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert len(got[0]) == 128 and got[0][:5] == bytes([0, 7, 0, 0, 255])
    assert got[1] == got[0] and got[2] == got[0]


def test_deadline_ends_a_stalled_wait():
    """dist.Deadline: a blocking call (RCCL init, a collective) that does not return in time
    ends the process with exit code 3 and a message naming the wait — a multi-GPU run with a
    missing peer fails fast instead of hanging."""
    code = ("import time\nfrom tf_image_compression_amd import dist\n"
            "with dist.Deadline('ncclCommInitRank (world 8)', 0.5, rank=5):\n    time.sleep(30)\n")
    env = {k: v for k, v in os.environ.items() if not k.startswith("TIC_DIST_")}  # 
    env["PYTHONPATH"] = ROOT
    env["TIC_DIST_TIMEOUT"] = "600"  # an explicit bound wins over the init-bound override
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=60, env=env)
    assert r.returncode == 3
    assert "[rank 5] ncclCommInitRank (world 8) did not complete within 0 s" in r.stderr or \
        "[rank 5] ncclCommInitRank (world 8) did not complete within 1 s" in r.stderr
    ok = subprocess.run([sys.executable, "-c", "from tf_image_compression_amd import dist\n"
                         "with dist.Deadline('x', 5.0, rank=0):\n    pass\nprint('done')"],
                        cwd=ROOT, capture_output=True, text=True, timeout=60, env=env)
    assert ok.returncode == 0 and ok.stdout.strip() == "done"


def _run_late(tmp_path, env_extra):
    port = _free_port()
    out = str(tmp_path / "late")
    env = {k: v for k, v in os.environ.items() if not k.startswith("TIC_DIST_")}
    env.update(PYTHONPATH=ROOT, OMP_NUM_THREADS="1", LATE_S="4", **env_extra)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "tests", "dist_worker.py"),
           out, "0", "0", "late"]
    r = subprocess.run(cmd, env=env, timeout=120, cwd=ROOT, capture_output=True, text=True)
    return r, out


def test_late_peer_within_collective_bound(tmp_path):
    """a collective also waits for its peers to arrive, and a peer may arrive late
    after rank-dependent work (tuning on one rank).  Rank 1 reaches its first collective 4 s
    after the start-up barrier; with a 2 s init bound that run must still pass (collectives
    have their own, longer bound), and dist.all_ranks gives every rank the same decision."""
    r, out = _run_late(tmp_path, {"TIC_DIST_TIMEOUT": "2"})
    assert r.returncode == 0, r.stderr[-2000:]
    res = [json.load(open(f"{out}.{k}")) for k in range(2)]
    assert [x["all_ranks"] for x in res] == [False, False] and all(x["all_true"] for x in res)


def test_step_collective_keeps_short_bound(tmp_path):
    """only collectives that follow rank-dependent work take the long bound (the
    caller passes it; dist.all_ranks does); a per-step collective keeps the short default
    (TIC_DIST_STEP_TIMEOUT), so a peer that stalls in the steady state ends the job quickly:
    with the late arrival at a plain barrier and a 1 s step bound, rank 0 exits with code 3."""
    r, _ = _run_late(tmp_path, {"TIC_DIST_STEP_TIMEOUT": "1", "LATE_AT": "barrier"})
    assert r.returncode != 0
    assert "gloo barrier did not complete within 1 s" in r.stderr


def test_late_peer_beyond_collective_bound(tmp_path):
    """The same late arrival with the collective bound set under it: rank 0 ends with exit
    code 3 and names the wait instead of hanging."""
    r, _ = _run_late(tmp_path, {"TIC_DIST_COLLECTIVE_TIMEOUT": "1"})
    assert r.returncode != 0
    assert "gloo all_reduce(max) did not complete within 1 s" in r.stderr
