"""bench.py's multi-rank launch on the CPU (gloo): ``python bench.py --gpus N`` without a
torchrun environment must start N ranks itself, each rank must agree on the world size and
its z-slab of the ONE strong-scaling grid, and the padded all-gather must reassemble every
plane once and in order (``--dry-run`` replaces the HIP kernel, which needs a GPU, by a fill
with the global plane index).  A world size that differs from ``--gpus`` must fail loudly."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def _env():
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env["OMP_NUM_THREADS"] = "1"
    return env


def _json_line(out):
    lines = [l for l in out.splitlines() if l.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


@pytest.mark.parametrize("n,grid", [(2, 24), (3, 20)])
def test_gpus_flag_spawns_ranks(n, grid):
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--dry-run",
                        "--grid", str(grid), "--particles", "3000"], cwd=ROOT, env=_env(),
                       capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout + r.stderr
    line = _json_line(r.stdout)
    assert line["n_gpus"] == n and line["world_size"] == n and line["gpus_flag"] == n
    from ptv_interpolation_amd import zslab

    assert line["partition"] == [list(zslab.rank_slab(grid, n, i)) for i in range(n)]
    # contiguous, covering, as even as possible
    edges = [p[0] for p in line["partition"]] + [line["partition"][-1][1]]
    assert edges[0] == 0 and edges[-1] == grid and all(a < b for a, b in zip(edges, edges[1:]))
    assert max(b - a for a, b in line["partition"]) - min(b - a for a, b in line["partition"]) <= 1
    assert line["particles_agree"] and line["field_reassembled"]
    # the warmup re-cut: every rank derives the same boundaries from the all-gathered step times,
    # and they even out the (synthetic) cost
    bal = line["balanced"]
    assert bal["ranks_agree"] and bal["bounds"][0] == 0 and bal["bounds"][-1] == grid
    assert all(a < b for a, b in zip(bal["bounds"], bal["bounds"][1:]))
    assert bal["cost_spread"][-1] <= bal["cost_spread"][0]


def test_world_size_mismatch_fails_loudly():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=2",
                        "--master-addr=127.0.0.1", f"--master-port={port}", os.path.join(ROOT, "bench.py"),
                        "--gpus", "3", "--dry-run", "--grid", "16", "--particles", "500"],
                       cwd=ROOT, env=_env(), capture_output=True, text=True, timeout=240)
    assert r.returncode != 0
    assert "--gpus 3 but the world size is 2" in r.stdout + r.stderr


def test_share_and_world_checks():
    import bench

    assert bench.parse_share("3/8") == (3, 8)
    for bad in ("8/8", "x/2", "1"):
        with pytest.raises(SystemExit):
            bench.parse_share(bad)

    class A:
        gpus = 4

    with pytest.raises(SystemExit):
        bench.check_world(A(), 2)
    bench.check_world(A(), 4)
    A.gpus = None
    bench.check_world(A(), 8)  # no --gpus: the launcher's world size stands
    # the default headline is strong scaling of the ONE named grid; weak stacking is opt-in
    assert bench.CONFIGS["headline"]["scaling"] == "strong"
    assert bench.CONFIGS["headline_weak"]["scaling"] == "weak"


def test_balanced_bounds_evens_out_the_cost():
    """zslab.balanced_bounds: a cut of the measured cost at k/N of the total, at least min_planes per
    slab, boundaries strictly increasing and covering the grid."""
    from ptv_interpolation_amd import zslab

    nz, n = 512, 8
    dens = [1.0 + (1.5 if 128 <= z < 200 or 320 <= z < 384 else 0.0) for z in range(nz)]
    b = [nz * r // n for r in range(n + 1)]
    spreads = []
    for _ in range(3):
        t = [sum(dens[b[r]:b[r + 1]]) for r in range(n)]
        spreads.append(max(t) / min(t))
        b = zslab.balanced_bounds(b, t)
        assert b[0] == 0 and b[-1] == nz and all(y - x >= 12 for x, y in zip(b, b[1:]))
    t = [sum(dens[b[r]:b[r + 1]]) for r in range(n)]
    assert max(t) / min(t) < 1.1 < spreads[0]
    assert zslab.balanced_bounds([0, 10, 20], [1.0]) == [0, 10, 20]  # mismatched input: unchanged
