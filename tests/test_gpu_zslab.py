"""GPU parity of the multi-GPU z-slab partition with replicated particles (SURVEY.md §8(e);
ptv_interpolation_amd/zslab.py; ptv_knn_params.slab_halo) and of one rank's share of the
BASELINE C4 / C5 configurations, against the oracle (scipy KDTree + numpy restatement of
interpolator.py:126-155, main.py:195-207 and physics.py:6-53).

A culled call bins fewer particles and so builds a different cell grid; that only reorders
candidates at exactly equal distances, so the results must equal the reference bit for bit
except at tie voxels (k-th and (k+1)-th neighbours equidistant) whose tied particles carry
different values; only those are excluded (tests/_util.hetero_ties), and their fraction is
printed.
"""
import numpy as np
import pytest

from tests._util import hetero_ties, hetero_ties_points

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from ptv_interpolation_amd import _lib

    if _lib.device_count() < 1:
        pytest.fail("no GPU visible: the gpu tests must run on an MI355X")
    return _lib.Context.get(0)


def _dev_cols(P, Q):
    import torch

    return [torch.from_numpy(np.ascontiguousarray(P[:, i])).cuda() for i in range(3)] + \
           [torch.from_numpy(np.ascontiguousarray(Q[:, i])).cuda() for i in range(3)]


def test_fluid_mask_device_matches_host():
    import torch

    from ptv_interpolation_amd import synth

    G = 96
    a = synth.fluid_mask(G).astype(np.uint8)
    b = synth.fluid_mask_device(G, 0, 2 * G, torch.device("cuda", 0)).cpu().numpy()
    assert np.array_equal(b[:G], a) and np.array_equal(b[G:], a)


def test_slab_cull_matches_whole_grid(ctx):
    """Four slabs of one grid, each from the replicated set with the cull: a tiny first halo is
    refused (InexactError with the proven halo), the retry is exact and bins fewer particles."""
    import torch

    from ptv_interpolation_amd import _lib, synth, zslab

    G = 64
    P, Q = synth.sphere_pack(40000, G, values="normal")
    cols = _dev_cols(P, Q)
    ax = torch.linspace(0, G - 1, G, dtype=torch.float64, device="cuda")
    ptrs = [c.data_ptr() for c in cols]
    whole = [torch.empty((G, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
    ctx.interp_knn_dev(len(P), ptrs, G, G, G, axes_ptrs=[ax.data_ptr()] * 3, out_ptrs=[o.data_ptr() for o in whole],
                       k=8)
    with pytest.raises(_lib.InexactError) as ei:
        slab = [torch.empty((16, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
        ctx.interp_knn_dev(len(P), ptrs, G, G, G, axes_ptrs=[ax.data_ptr()] * 3,
                           out_ptrs=[o.data_ptr() for o in slab], k=8, z_range=(16, 32), slab_halo=0.25)
    assert ei.value.halo_required > 0.25
    binned = []
    for z0, z1 in zslab.slab_bounds(G, 4):
        slab = [torch.empty((z1 - z0, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
        state = zslab.HaloState(0.25)

        def call(h):
            return ctx.interp_knn_dev(len(P), ptrs, G, G, G, axes_ptrs=[ax.data_ptr()] * 3,
                                      out_ptrs=[o.data_ptr() for o in slab], k=8, z_range=(z0, z1), slab_halo=h)

        zslab.interp_slab(call, state)
        st = ctx.last_stats()
        assert state.retries >= 1 and st["halo_required"] <= state.halo
        binned.append(st["n_binned"])
        axh = np.linspace(0, G - 1, G)
        tie, het = hetero_ties(P, Q, axh, axh, axh[z0:z1], 8)
        print(f"slab [{z0}, {z1}): ties {tie.mean():.4%}, value-heterogeneous (excluded) {het.mean():.4%}")
        for a, b in zip(slab, whole):
            a, b = a.cpu().numpy(), b[z0:z1].cpu().numpy()
            assert np.array_equal(a[~het], b[~het])
    assert min(binned) < len(P)


@pytest.mark.timeout(500)
def test_c4_rank_share_masked_with_boundary_particles():
    """C4 (BASELINE configs[3]): 1024^3 grid / 10M sphere-pack particles + the pore-mask path
    (extract_boundary_particles, every 4th boundary voxel, zero velocity) + the fused
    main.py:195-207 epilogue; rank 2 of 8 (planes 256..383, cutting through the lower
    spheres) on the replicated set through the shipped N > 1 path (bench.py): the per-column cull
    map of PTV_FLAG_SLAB_CULL_AUTO on a fresh context, one cold call (every particle binned, the
    map built) and one warm call (culled, proven on the device); both against the oracle on 20k
    sampled voxels."""
    import json
    import time

    import torch

    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib, synth, zslab
    from ptv_interpolation_amd import interpolator as ip

    G, n, world, rank = 1024, 10_000_000, 8, 2
    P, Q = synth.sphere_pack(n, G, values="normal")
    fluid_d = synth.fluid_mask_device(G, 0, G, torch.device("cuda", 0))
    fluid = fluid_d.cpu().numpy().view(bool)
    bx, by, bz = ip.extract_boundary_particles(fluid, ((0, G),) * 3, sampling_step=4, thickness=1)
    P = np.concatenate([P, np.stack([bx, by, bz], 1)])
    Q = np.concatenate([Q, np.zeros((len(bx), 3))])
    cols = _dev_cols(P, Q)
    ax = torch.linspace(0, G - 1, G, dtype=torch.float64, device="cuda")
    z0, z1 = zslab.rank_slab(G, world, rank)
    rng = np.random.default_rng(4)
    sel = rng.integers(0, (z1 - z0) * G * G, 20000)
    iz, iy, ix = np.unravel_index(sel, (z1 - z0, G, G))
    q = np.stack([ix, iy, iz + z0], -1).astype(np.float64)
    ref = cpu_ref.interp_points(P, Q, q, "idw", 8, 2.0)
    solid = ~fluid[iz + z0, iy, ix]
    ref[solid] = 0.0
    ref = np.nan_to_num(ref)
    tie, het = hetero_ties_points(P, Q, q, 8)
    het &= ~solid  # solid voxels are written as 0 whatever their neighbours
    print(f"C4 rank share: ties {tie.mean():.4%} of sampled voxels, value-heterogeneous (excluded) {het.mean():.4%}")
    assert het.mean() < 0.01
    ctx = _lib.Context(0)  # fresh: no cached cull map
    out = [torch.empty((z1 - z0, G, G), dtype=torch.float64, device="cuda") for _ in range(3)]
    try:
        for call in ("cold", "warm"):
            for o in out:
                o.fill_(-7.0)
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            ctx.interp_knn_dev(len(P), [c.data_ptr() for c in cols], G, G, G, axes_ptrs=[ax.data_ptr()] * 3,
                               out_ptrs=[o.data_ptr() for o in out], k=8, mask_ptr=fluid_d.data_ptr(),
                               flags=_lib.FLAG_NAN_TO_NUM | _lib.FLAG_SLAB_CULL_AUTO, z_range=(z0, z1))
            torch.cuda.synchronize()
            wall = (time.perf_counter() - t0) * 1e3
            st = ctx.last_stats()
            print("SHARE " + json.dumps({"config": "c4", "rank": rank, "world": world, "planes": [z0, z1],
                                         "call": call, "wall_ms": round(wall, 3),
                                         "device_ms": round(st["ms_bin"] + st["ms_cull"] + st["ms_lattice"] +
                                                            st["ms_knn"], 3),
                                         "n_binned": int(st["n_binned"]), "n_particles": len(P)}))
            assert (st["n_binned"] == len(P)) if call == "cold" else (st["n_binned"] < len(P))
            got = [o.reshape(-1)[torch.from_numpy(sel).cuda()].cpu().numpy() for o in out]
            for c in range(3):
                assert np.array_equal(got[c][~het], ref[~het, c])
    finally:
        ctx.close()


@pytest.mark.timeout(600)
def test_c5_rank_share_f32_and_divergence(ctx):
    """C5 (BASELINE configs[4]): 2048^3 grid / 50M particles, float32 field
    (PTV_FLAG_OUT_F32 = the fused main.py:230 astype), rank 3 of 8 (planes 768..1023, through
    the lower spheres' voids) plus one redundantly interpolated halo plane per side, then the
    float32 consistent divergence of the slab (physics.py:6-53, view_divergence.py:39).
    20k sampled voxels against astype(float32) of the f64 oracle; two planes of the divergence
    against the oracle divergence of the GPU field."""
    import torch

    from oracle import cpu_ref
    from ptv_interpolation_amd import _lib, synth, zslab
    from scipy.spatial import KDTree

    G, n, world, rank = 2048, 50_000_000, 8, 3
    P, Q = synth.sphere_pack(n, G, values="normal")
    cols = _dev_cols(P, Q)
    ax = torch.linspace(0, G - 1, G, dtype=torch.float64, device="cuda")
    z0, z1 = zslab.rank_slab(G, world, rank)
    za, zb, hlo, hhi = zslab.halo_slab(z0, z1, G, 1)
    out = [torch.empty((zb - za, G, G), dtype=torch.float32, device="cuda") for _ in range(3)]
    state = zslab.HaloState(zslab.halo_guess(n, (G, G, G), 8))

    def call(h):
        return ctx.interp_knn_dev(n, [c.data_ptr() for c in cols], G, G, G, axes_ptrs=[ax.data_ptr()] * 3,
                                  out_ptrs=[o.data_ptr() for o in out], k=8, flags=_lib.FLAG_OUT_F32,
                                  z_range=(za, zb), slab_halo=h)

    zslab.interp_slab(call, state)
    assert ctx.last_stats()["n_binned"] < n
    mask = synth.fluid_mask_device(G, za, zb, torch.device("cuda", 0))
    torch.cuda.synchronize()  # the mask comes from torch's stream, the divergence runs on the context's
    div = torch.empty((z1 - z0, G, G), dtype=torch.float32, device="cuda")
    ctx.divergence_dev(G, G, zb - za, [o.data_ptr() for o in out], mask.data_ptr(), div.data_ptr(), 1.0, 1.0, 1.0,
                       field_dtype=_lib.F32, result_dtype=_lib.F32, z_range=(hlo, hlo + (z1 - z0)),
                       edges=(hlo == 0, hhi == 0))
    torch.cuda.synchronize()
    del cols
    # oracle: a KDTree over the particles within H of the slab; every sampled voxel's k-th
    # distance is checked to be <= H + its distance to the nearer slab face (then no particle
    # outside the subset can be among its k nearest: the oracle is exact for it)
    H = 320.0
    keep = (P[:, 2] >= za - H) & (P[:, 2] <= zb - 1 + H)
    Ps, Qs = P[keep], Q[keep]
    del P, Q
    rng = np.random.default_rng(5)
    sel = rng.integers(0, (zb - za) * G * G, 20000)
    iz, iy, ix = np.unravel_index(sel, (zb - za, G, G))
    q = np.stack([ix, iy, iz + za], -1).astype(np.float64)
    tree = KDTree(Ps)
    d, _ = tree.query(q, k=9, workers=-1)
    m = np.minimum(q[:, 2] - (za - H), (zb - 1 + H) - q[:, 2])
    assert (d[:, 7] < m).all()
    ties = d[:, 7] == d[:, 8]  # continuous N(0,1) values: every tie is value-heterogeneous
    print(f"C5 rank share: ties (excluded) {ties.mean():.4%} of sampled voxels")
    assert ties.mean() < 0.01
    ref = cpu_ref.interp_points(Ps, Qs, q, "idw", 8, 2.0).astype(np.float32)
    tsel = torch.from_numpy(sel).cuda()
    for c in range(3):
        got = out[c].reshape(-1)[tsel].cpu().numpy()
        assert np.array_equal(got[~ties], ref[~ties, c])
    # divergence: planes 0 (reads the lower halo plane) and 128 of the slab
    for p in (0, 128):
        b = hlo + p  # buffer plane
        blk = [o[b - 1:b + 2].cpu().numpy() for o in out]
        mk = mask[b - 1:b + 2].cpu().numpy().view(bool)
        exp = cpu_ref.consistent_divergence(blk[0], blk[1], blk[2], mk, 1.0, 1.0, 1.0)[1]
        assert exp.dtype == np.float32
        assert np.array_equal(div[p].cpu().numpy(), exp, equal_nan=True)
