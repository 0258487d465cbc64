#!/usr/bin/env python3
"""Two node-sharded engines, one process each, exchanging published
preferences with RCCL (av_comm_init + ncclAllGather every round), compared bit
for bit with a single unsharded engine. On a 1-GPU box both ranks use device
0, which RCCL may refuse; the script then says so and exits 3.

    python tools/rccl_two_rank_probe.py
"""
import os
import sys
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "go-avalanche_amd", "python"))

N, M, K, R = 64, 200, 8, 20
BYZ = int(0.2 * 2**32)


def rank_main(rank, uid_path, out_dir, q):
    import torch  # noqa: F401

    import avhip

    try:
        with open(uid_path, "rb") as f:
            uid = f.read()
        e = avhip.Engine(N, M, k=K, seed=9, byz_threshold=BYZ, node_range=(rank * N // 2, (rank + 1) * N // 2),
                         device=0)
        e.init_records(avhip.INIT_PAIRS, 0)
        e.comm_init(2, rank, uid)
        e.run_rounds(R)
        np.save(os.path.join(out_dir, f"rec{rank}.npy"), e.read_records())
        np.save(os.path.join(out_dir, f"upd{rank}.npy"), e.fetch_updates())
        q.put((rank, "ok"))
    except Exception as ex:  # report, do not hang the parent
        q.put((rank, f"error: {ex}"))


def main():
    import multiprocessing as mp

    import torch  # noqa: F401

    import avhip

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with tempfile.TemporaryDirectory() as d:
        uid_path = os.path.join(d, "uid")
        with open(uid_path, "wb") as f:
            f.write(avhip.comm_unique_id())
        procs = [ctx.Process(target=rank_main, args=(r, uid_path, d, q)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=150)
        for p in procs:
            if p.is_alive():
                p.kill()
                print("probe: rank hung (killed)")
                sys.exit(3)
        res = dict(q.get() for _ in range(2))
        if any(v != "ok" for v in res.values()):
            print("probe: RCCL refused two ranks on one device:", res)
            sys.exit(3)
        ref = avhip.Engine(N, M, k=K, seed=9, byz_threshold=BYZ)
        ref.init_records(avhip.INIT_PAIRS, 0)
        ref.run_rounds(R)
        rec = np.concatenate([np.load(os.path.join(d, f"rec{r}.npy")) for r in range(2)])
        upd = np.concatenate([np.load(os.path.join(d, f"upd{r}.npy")) for r in range(2)])
        upd = upd[np.lexsort((upd[:, 3], upd[:, 2], upd[:, 1], upd[:, 0]))]
        ok = np.array_equal(rec, ref.read_records()) and np.array_equal(upd, ref.fetch_updates())
        print("probe: 2-rank node-sharded RCCL engine", "== single engine (bit-exact)" if ok else "MISMATCH")
        sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
