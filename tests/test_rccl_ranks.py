"""Two and four RCCL ranks exchanging through libbpgl's own communicator (column shards: the reference's
P-way split, cpu_calculation.py:23-27 / lasso.py:101-126; row shards: one feature block).

The ranks run on the one GPU of the test box as separate processes under torch.distributed.run,
each announcing its own NCCL_HOSTID so RCCL accepts them (the all-reduce then crosses loopback
sockets instead of xGMI: correctness only, no timing).  Unlike tests/test_rowshard.py, whose
multi-rank cases sum the exchange buffers in the test, here the product's ncclAllReduce (inside
the captured graph and eager) is the exchange.  Row shards on a shared GPU cannot keep the
one-pass kernel's blocks co-resident unless every rank's stream is confined to its own CUs:
without CU masks they normally finish on the two-pass row iteration;
with XCD-symmetric CU masks (``--cumask``: 2 ranks x 128 CUs, 4 x 64, 8 x 32) each rank's
persistent grid is sized to its CUs and the default N > 1 path -- one-pass row shards, k_onepass
+ k_onepass_fold + ncclAllReduce of [U | r.s23 | s23.s23 | failed] + k_onepass_tail -- runs
end to end with no fallback.  Tolerance: the reference fixture's x within 1e-9 relative l2
(as every solver test), the ranks' x bit-identical (rows), graph = eager.
"""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")
if not torch.cuda.is_available():
    pytest.skip("no GPU", allow_module_level=True)

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(case, shard, tmp_path, world=2, extra=(), timeout=240):
    env = dict(os.environ)
    env.pop("NCCL_HOSTID", None)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "tests", "rccl_ranks_worker.py"), case, shard, str(tmp_path), *extra]
    p = subprocess.run(cmd, env=env, cwd=ROOT, capture_output=True, text=True, timeout=timeout)
    assert p.returncode == 0, p.stdout[-3000:] + p.stderr[-3000:]
    return [dict(np.load(tmp_path / f"rank{r}.npz")) for r in range(world)]


def rel(a, b):
    a, b = np.asarray(a).reshape(-1), np.asarray(b).reshape(-1)
    return np.linalg.norm(a - b) / max(np.linalg.norm(b), 1e-300)


@pytest.mark.parametrize("case,world", [("c1_b2_p4_f32in", 2), ("bound_b4_p2_f32in", 2), ("c1_b2_p4_f32in", 4),
                                        ("c1_b2_p4_f32in", 8), ("randbound231_b4_p2_f32in", 2),
                                        ("randbound545_b4_p1_f32in", 4), ("raggedbound74_b3_p2_f32in", 2)])
def test_two_rccl_ranks_column_shards(golden, case, world, tmp_path):
    from convex_optimization_amd import distributed as D
    fx = golden(case)
    out = _launch(case, "columns", tmp_path, world)
    for tag in ("graph", "eager"):
        x = D.assemble_x([o[f"x_{tag}"] for o in out], int(fx["BLOCK"]))
        assert rel(x, fx["x"]) <= 1e-9, (tag, rel(x, fx["x"]))
        for o in out:
            assert int(o[f"t_last_{tag}"]) == int(fx["t_last"]) and bool(o[f"stopped_{tag}"]) == bool(fx["stopped"])
        T = int(fx["t_last"]) + 1
        np.testing.assert_allclose(out[0][f"err_{tag}"][:T], fx["err_iter"][:T], rtol=1e-6, atol=1e-9)
        for o in out[1:]:
            np.testing.assert_array_equal(out[0][f"err_{tag}"][:T], o[f"err_{tag}"][:T])
    np.testing.assert_array_equal(out[0]["x_graph"], out[0]["x_eager"])


@pytest.mark.parametrize("world", [2, 4])
def test_two_rccl_ranks_row_shards(golden, world, tmp_path):
    fx = golden("c1_b1_p1_f32in")
    out = _launch("c1_b1_p1_f32in", "rows", tmp_path, world)
    for o in out[1:]:
        np.testing.assert_array_equal(out[0]["diag"], o["diag"])      # all-reduced column norms
    np.testing.assert_allclose(out[0]["diag"], fx["d_ATA"].reshape(-1), rtol=1e-12)
    for tag in ("graph", "eager"):
        for o in out[1:]:
            np.testing.assert_array_equal(out[0][f"x_{tag}"], o[f"x_{tag}"])   # x replicated bit for bit
        assert rel(out[0][f"x_{tag}"], fx["x"]) <= 1e-9, (tag, rel(out[0][f"x_{tag}"], fx["x"]))
        T = int(fx["ITER_MAX"])
        np.testing.assert_allclose(out[0][f"err_{tag}"][:T], fx["err_iter"][:T], rtol=1e-6, atol=1e-9)
    print("row-shard fallbacks per rank:", [int(o["fallbacks"]) for o in out])


@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_row_shards_onepass_cu_masked(golden, world, tmp_path):
    """The default N > 1 iteration (one-pass row shards over RCCL), every rank on its own CUs:
    no rank falls back, x is bit-identical on every rank and matches the reference fixture
    (c1_b1_p1_f32in: the reference's ClassLassoCPU on the fp32-rounded instance, lasso.py:102-157,
    whose P-way shard sum lasso.py:107-126 is here a sum over ranks)."""
    fx = golden("c1_b1_p1_f32in")
    out = _launch("c1_b1_p1_f32in", "rows", tmp_path, world, ["--cumask"])
    cus = torch.cuda.get_device_properties(0).multi_processor_count
    for o in out:
        assert int(o["cus"]) == cus // world and int(o["cu_masked"]) == 1, (o["cus"], o["cu_masked"])
        assert 0 < int(o["onepass_grid"]) <= cus // world
    for tag in ("graph", "eager"):
        for o in out:
            assert int(o[f"onepass_{tag}"]) == 1 and int(o[f"fallbacks_{tag}"]) == 0, \
                (tag, int(o[f"onepass_{tag}"]), int(o[f"fallbacks_{tag}"]))
        for o in out[1:]:
            np.testing.assert_array_equal(out[0][f"x_{tag}"], o[f"x_{tag}"])
        assert rel(out[0][f"x_{tag}"], fx["x"]) <= 1e-9, (tag, rel(out[0][f"x_{tag}"], fx["x"]))
        T = int(fx["ITER_MAX"])
        np.testing.assert_allclose(out[0][f"err_{tag}"][:T], fx["err_iter"][:T], rtol=1e-6, atol=1e-9)
    np.testing.assert_array_equal(out[0]["x_graph"], out[0]["x_eager"])


@pytest.mark.parametrize("case,world", [("stop511_b1_p1_f32in", 2), ("stop257_b1_p4_f32in", 4),
                                        ("stop513_b1_p4_f32in", 2)])
def test_rccl_row_shards_stop_rule_pinned(golden, case, world, tmp_path):
    """ERR_BOUND on one-pass row shards over RCCL (each rank on its own CUs): the error criterion
    comes from the all-reduced carried g, and the stop iteration must be the reference's own
    (ClassLassoCPU, lasso.py:141-150) on every rank, in graph replay and eager, with no fallback."""
    fx = golden(case)
    out = _launch(case, "rows", tmp_path, world, ["--cumask"])
    T = int(fx["t_last"])
    for tag in ("graph", "eager"):
        for o in out:
            assert int(o[f"onepass_{tag}"]) == 1 and int(o[f"fallbacks_{tag}"]) == 0
            assert int(o[f"t_last_{tag}"]) == T and bool(o[f"stopped_{tag}"]), (tag, int(o[f"t_last_{tag}"]), T)
        for o in out[1:]:
            np.testing.assert_array_equal(out[0][f"x_{tag}"], o[f"x_{tag}"])
        assert rel(out[0][f"x_{tag}"], fx["x"]) <= 1e-9, (tag, rel(out[0][f"x_{tag}"], fx["x"]))
        np.testing.assert_allclose(out[0][f"err_{tag}"][:T + 1], fx["err_iter"][:T + 1], rtol=1e-6)


def test_rccl_row_shards_collective_recovery(golden, tmp_path):
    """One rank's one-pass launch fails (test hook on rank 0 only, inside an 8-iteration graph):
    its flag rides the all-reduce, every rank skips the same iterations, and every rank's
    bpgl_solver_status (entered concurrently, one process per rank) re-runs them on the two-pass
    row iteration -- the same fallback count and the same x on every rank, the reference's x."""
    fx = golden("c1_b1_p1_f32in")
    out = _launch("c1_b1_p1_f32in", "rows", tmp_path, 2, ["--cumask", "--fail-rank", "0", "--fail-at", "37"])
    for o in out:
        assert int(o["fallbacks_graph"]) == 1 and int(o["onepass_graph"]) == 0
        assert int(o["fallbacks_eager"]) == 0 and int(o["onepass_eager"]) == 1
    for tag in ("graph", "eager"):
        np.testing.assert_array_equal(out[0][f"x_{tag}"], out[1][f"x_{tag}"])
        assert rel(out[0][f"x_{tag}"], fx["x"]) <= 1e-9, (tag, rel(out[0][f"x_{tag}"], fx["x"]))


def _one_gpu_x(fx, iters):
    """x after `iters` iterations of the single-GPU product path on the fixture's hash instance
    (tests/test_longrun.py holds that path to the C oracle's fixture over the whole horizon)"""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import hash_instance as H
    from convex_optimization_amd.gpu_calculation import GPU_Calculation
    m, n = int(fx["m"]), int(fx["n"])
    A = H.torch_A(m, n, "cuda:0")
    b = H.torch_b(A, row0=0, m_total=m)
    gc = type("GC_float", (GPU_Calculation,), {"TYPE": "float"})(A, 1, device=0)
    x = gc.run(b, float(fx["mu"]), iters)["x"]
    del gc, A, b
    torch.cuda.empty_cache()
    return x


@pytest.mark.timeout(900)
@pytest.mark.parametrize("world", [2, 4, 8])
def test_rccl_row_shards_configs2_long_horizon(world, tmp_path):
    """configs[2] (8192 x 524288 fp32, 16 GiB) over WORLD RCCL row ranks on one GPU, each on its own
    1/WORLD of the CUs, against the C oracle's fixture (tests/golden/longrun_configs2.npz, hash
    instance, the reference's ITER_MAX = 1000 iterations, cpu_vs_gpu.py:66): x within north_star's
    1e-5 relative l2 and the error-criterion trace as tests/test_longrun.py, x bit-identical on
    every rank, no fallback.

    World 2 (4096 x 524288 per rank on 128 CUs) runs the default one-pass row iteration: 128 segment
    blocks per row (two hand-off granules per lane, as the N = 8 weak leg's shard on an 8-GPU node),
    one ncclAllReduce of 4 MiB + 4 words per iteration, three exact-gradient refreshes.  Worlds 4
    and 8 cannot run it on ONE GPU: a row of 524288 fp32 columns needs 128 co-resident segment
    blocks (one per CU), more than a 64- or 32-CU partition holds (on an 8-GPU node every rank has
    256 CUs).  They run the two-pass row iteration instead (exact g = sum_q A_q^T r_q through an
    all-reduce of w, s23 = A_q D on the local rows, an all-reduce of the line-search scalars): the
    same 4- and 8-rank RCCL exchange at full size.  World 8 runs the fixture's first 300 iterations
    (two 4 MiB loopback all-reduces per iteration among 8 processes): its error-criterion trace is
    held to the fixture's first 300 entries and its x to the single-GPU product path's x after the
    same 300 iterations (tests/test_longrun.py holds that path to the fixture over 1000)."""
    path = os.path.join(ROOT, "tests", "golden", "longrun_configs2.npz")
    fx = dict(np.load(path))
    IT = int(fx["iters"]) if world < 8 else 300
    out = _launch("longrun_configs2", "rows", tmp_path, world, ["--cumask", "--iters", str(IT)], timeout=840)
    onepass = world == 2
    for o in out:
        assert bool(o["samples_ok"]) and bool(o["b_ok"]) and bool(o["in_place"])
        assert int(o["iters"]) == IT
        assert int(o["onepass"]) == int(onepass) and int(o["fallbacks"]) == 0, (int(o["onepass"]), int(o["fallbacks"]))
        assert int(o["refreshes"]) == ((IT - 1) // 256 if onepass else 0)
    for o in out[1:]:
        np.testing.assert_array_equal(out[0]["x"], o["x"])
    ref = fx["err_iter"][:IT]
    np.testing.assert_allclose(out[0]["err"][:IT], ref, rtol=1e-4, atol=1e-6 * ref[0])
    if IT == int(fx["iters"]):
        e = rel(out[0]["x"], fx["x"])
        what = "the C oracle"
    else:
        e = rel(out[0]["x"], _one_gpu_x(fx, IT))
        what = "the one-GPU product path"
        assert e <= 1e-8, e
    print(f"configs2 over {world} RCCL row ranks ({int(out[0]['cus'])} CUs each, "
          f"{'one pass' if onepass else 'two passes'}), {IT} iterations: rel l2 vs {what} {e:.3e}")
    assert e <= 1e-5, e


@pytest.mark.timeout(600)
@pytest.mark.parametrize("world,fp32", [(4, False), (4, True), (8, True)])
def test_rccl_row_shards_configs1_long_horizon_exchange(world, fp32, tmp_path):
    """configs[1] (8192 x 65536 fp32) over 4 and 8 RCCL row ranks on one GPU's CU partitions (2048 /
    1024 rows per rank: 16 segment blocks, one pass), against the C oracle's fixture
    (tests/golden/longrun_configs1.npz): with the default fp64 exchange and with the opt-in fp32 one
    (U rounded to fp32 per rank before the cross-rank sum, the line-search scalars as hi + lo pairs;
    half the all-reduce bytes).  World 4 runs the reference's 1000 iterations (x against the oracle);
    world 8 the first 300 (x against the single-GPU product path after the same 300 iterations),
    enqueued 8 iterations (one captured graph) at a time with the stream drained in between: eight
    processes on ONE GPU exchanging over loopback sockets stalled when all 300 were enqueued at once
    (profiles/r06/check_g; the bench's N > 1 legs drain every window too, and on an 8-GPU node each
    rank has its own device).  All within north_star's 1e-5 on x -- the measurement behind keeping
    fp64 the default."""
    fx = dict(np.load(os.path.join(ROOT, "tests", "golden", "longrun_configs1.npz")))
    IT = int(fx["iters"]) if world <= 4 else 300
    extra = ["--cumask", "--iters", str(IT)] + (["--exchange-fp32"] if fp32 else []) + \
        (["--chunk", "8"] if world == 8 else [])
    out = _launch("longrun_configs1", "rows", tmp_path, world, extra, timeout=540)
    for o in out:
        assert bool(o["samples_ok"]) and bool(o["b_ok"]) and int(o["iters"]) == IT
        assert int(o["onepass"]) == 1 and int(o["fallbacks"]) == 0
    for o in out[1:]:
        np.testing.assert_array_equal(out[0]["x"], o["x"])
    ref = fx["err_iter"][:IT]
    np.testing.assert_allclose(out[0]["err"][:IT], ref, rtol=1e-3, atol=1e-6 * ref[0])
    if IT == int(fx["iters"]):
        e, what = rel(out[0]["x"], fx["x"]), "the C oracle"
    else:
        e, what = rel(out[0]["x"], _one_gpu_x(fx, IT)), "the one-GPU product path"
    print(f"configs1 over {world} RCCL row ranks, {'fp32' if fp32 else 'fp64'} exchange, {IT} iterations: "
          f"rel l2 vs {what} {e:.3e}")
    assert e <= 1e-5, e
