"""Worker for tests/test_dist.py (launched by torch.distributed.run, gloo, CPU only).

Runs the image-parallel shard loop of tf_image_compression_amd.sharded with the CPU
oracle standing in for the per-rank GPU codec, all-gathers the stats over gloo, and
(rank 0) writes the combined metrics + the exchanged RCCL-style unique id to a JSON file."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import tic_oracle as o  # noqa: E402
from tf_image_compression_amd import dist, sharded  # noqa: E402
from tf_image_compression_amd.weights import synthetic_params, SYNTH_MEAN, SYNTH_STD  # noqa: E402


def main():
    out, n_images, P = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
    driver = sys.argv[4] if len(sys.argv) > 4 else "host"
    comm = dist.make_comm()  # gloo at world > 1; one barrier under the init bound
    if driver == "late":  # rank 1 arrives at the next collective late (tuning on one rank)
        import time
        if comm.rank == 1:
            time.sleep(float(os.environ.get("LATE_S", "3")))
        if os.environ.get("LATE_AT") == "barrier":  # a per-step collective: the short default bound
            comm.barrier()
        ok = dist.all_ranks(comm, comm.rank == 0)
        with open(f"{out}.{comm.rank}", "w") as f:
            json.dump({"rank": comm.rank, "all_ranks": ok, "all_true": dist.all_ranks(comm, True)}, f)
        comm.close()
        return
    params = synthetic_params(1)

    if driver == "device":  # the GPU driver's orchestration (sharded.run_device_shard)
        sys.path.insert(0, os.path.join(ROOT, "tests"))
        from host_codec import HostCodec
        codec = HostCodec(1, params, SYNTH_MEAN, SYNTH_STD, P)
        _, st = sharded.run_device_shard(codec, comm, comm.rank, comm.world, n_images, batch=3)
        assert codec.calls == -(-st.images // 3)
    else:
        def codec_fn(x):
            _, idx = o.encoder(params, SYNTH_MEAN, SYNTH_STD, x, P, 2, 1)
            return o.decoder(params, SYNTH_MEAN, SYNTH_STD, idx, 2, 1)[1]

        st = sharded.run_shard(codec_fn, comm.rank, comm.world, n_images, P, 3, (P // 16) ** 2 * 64)
    stats = comm.allgather_stats(st)
    tmax = comm.allreduce_max(float(comm.rank + 1))
    # TCP bootstrap of the 128-byte RCCL unique id (same code path as RcclComm)
    port = int(os.environ["MASTER_PORT"]) + 17
    payload = bytes(range(128)) if comm.rank == 0 else None
    uid = dist.exchange_unique_id(comm.rank, comm.world, payload, "127.0.0.1", port)
    rows = comm.allgather_f64([comm.rank, 10 + comm.rank, 7.5])  # bench.py's per-rank device record path
    res = {"rank": comm.rank, "summary": dist.combine(stats), "tmax": tmax, "uid_ok": uid == bytes(range(128)),
           "images": [s.images for s in stats], "gather": rows.tolist()}
    with open(f"{out}.{comm.rank}", "w") as f:
        json.dump(res, f)
    comm.barrier()
    comm.close()


if __name__ == "__main__":
    main()
