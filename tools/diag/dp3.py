"""Diagnose DP-vs-single weight mismatches on the 1e8 murmur3 tiered case.

python tools/diag/dp3.py <world> <mode>   mode: prefetch | inline | noprep
Spawns <world> gloo ranks on GPU 0 (like tests/test_gpu_dp_procs.py), trains
the wide 1e8 case, then compares with a single engine and prints where the
weights differ.
"""
import os
import sys
import tempfile

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
import test_gpu_dp_procs as T  # noqa: E402

CASE = 2


def worker(rank, world, port, out_dir, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world), LOCAL_RANK=str(rank))
    import torch  # noqa: F401
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    from twitter_stream_ml_amd.parallel import dist as D
    D.init_distributed(backend="gloo")
    comm = D.make_comm(0, "gloo")
    keep = []
    for ci in (range(CASE + 1) if os.environ.get("DIAG_ALL") else [CASE]):   # DIAG_ALL: like the test
        profile, F, hash, rows, nb, _ = T.LR_CASES[ci]
        eng = DeviceLinearRegression(T._lr_cfg(F, hash, rows), device=0, comm=comm)
        shards = [full.shard(rank, world) for full in T._batches(profile, rows, nb, seed=40 + ci)]
        if mode == "prefetch":
            for sh in shards[:eng.raw_slots - 1]:
                eng.prefetch(sh)
        its = []
        for t, sh in enumerate(shards):
            r = eng.train_batch(sh, want_pred=False)
            its.append(r["iterations"])
            if ci == CASE:
                np.save(os.path.join(out_dir, f"w{rank}_{t}.npy"), eng.get_weights())
        if ci == CASE:
            np.save(os.path.join(out_dir, f"it{rank}.npy"), np.array(its))
        if os.environ.get("DIAG_KEEP"):
            keep.append(eng)
        del eng
        if os.environ.get("DIAG_GC"):
            import gc
            gc.collect()
    if os.environ.get("DIAG_GC_THREAD"):   # collect from inside every HostComm callback
        pass
    D.barrier()
    D.shutdown()


def main():
    world, mode = int(sys.argv[1]), sys.argv[2]
    import torch.multiprocessing as mp
    out = tempfile.mkdtemp()
    mp.start_processes(worker, args=(world, T._free_port(), out, mode), nprocs=world, join=True,
                       start_method="spawn")
    from twitter_stream_ml_amd.ops.lr_engine import DeviceLinearRegression
    profile, F, hash, rows, nb, _ = T.LR_CASES[CASE]
    single = DeviceLinearRegression(T._lr_cfg(F, hash, rows), device=0)
    single2 = DeviceLinearRegression(T._lr_cfg(F, hash, rows), device=0)
    for t, full in enumerate(T._batches(profile, rows, nb, seed=40 + CASE)):
        r1 = single.train_batch(full, want_pred=False)
        single2.train_batch(full, want_pred=False)
        w1 = single.get_weights()
        w2 = single2.get_weights()
        print(f"single vs single batch {t}: max diff {np.abs(w1 - w2).max():.3g}")
        scale = np.abs(w1).max()
        for rk in range(world):
            w = np.load(os.path.join(out, f"w{rk}_{t}.npy"))
            d = np.abs(w - w1)
            bad = d > 1e-4 * np.abs(w1) + 1e-6 * scale
            nz1, nz = np.count_nonzero(w1), np.count_nonzero(w)
            print(f"world {world} {mode} batch {t} rank {rk}: iters {r1['iterations']} vs "
                  f"{np.load(os.path.join(out, f'it{rk}.npy'))[t]}, nnz {nz1} vs {nz}, bad {bad.sum()}, "
                  f"max diff {d.max():.3g}")
            if bad.any() and rk == 0:
                idx = np.nonzero(bad)[0]
                o = np.argsort(-d[idx])[:8]
                for i in idx[o]:
                    print(f"   id {i}: single {w1[i]:.6g} dp {w[i]:.6g}")
                print("   zero in single:", int((w1[idx] == 0).sum()), "zero in dp:", int((w[idx] == 0).sum()),
                      "sign flips:", int((np.sign(w1[idx]) != np.sign(w[idx])).sum()))
        if t == 0:
            pass
    for rk in range(1, world):
        same = np.array_equal(np.load(os.path.join(out, f"w{rk}_{nb - 1}.npy")),
                              np.load(os.path.join(out, f"w0_{nb - 1}.npy")))
        print(f"replica {rk} == rank 0: {same}")


if __name__ == "__main__":
    main()
