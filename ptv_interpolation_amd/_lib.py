"""ctypes binding of the C ABI in include/ptv_api.h (libptv_amd.so, built in-tree).

The shipped path has no CPU fallback: if the library is missing or no GPU is
visible, ``lib()`` / ``Context`` raise.  Structures mirror the header field by
field.
"""
from __future__ import annotations

import ctypes as C
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
_DEFAULT_LIB = os.path.join(HERE, "libptv_amd.so")
LIB_PATH = os.environ.get("PTV_LIB", _DEFAULT_LIB)

PTV_OK = 0
PTV_E_ARG = -1
PTV_E_HIP = -2
PTV_E_NOMEM = -3
PTV_E_UNSUPPORTED = -4
PTV_E_INEXACT = -5
PTV_E_SINGULAR = -6

METHOD_IDW = 0
METHOD_SIBSON = 1
METHOD_NEAREST = 2
METHOD_IDW_RADIUS = 3  # extension: IDW over every particle within a radius (parity unpinned)

FLAG_NAN_TO_NUM = 1

# local RBF kernels (include/ptv_api.h PTV_RBF_*), scipy names
RBF_KERNELS = {
    "linear": 0,
    "thin_plate_spline": 1,
    "cubic": 2,
    "quintic": 3,
    "multiquadric": 4,
    "inverse_multiquadric": 5,
    "inverse_quadratic": 6,
    "gaussian": 7,
}

_dp = C.POINTER(C.c_double)


class Particles(C.Structure):
    _fields_ = [("n", C.c_int64), ("x", _dp), ("y", _dp), ("z", _dp), ("u", _dp), ("v", _dp), ("w", _dp)]


class Grid(C.Structure):
    _fields_ = [("nx", C.c_int64), ("ny", C.c_int64), ("nz", C.c_int64),
                ("ax", _dp), ("ay", _dp), ("az", _dp),
                ("px", _dp), ("py", _dp), ("pz", _dp),
                ("z_begin", C.c_int64), ("z_end", C.c_int64)]


class KnnParams(C.Structure):
    _fields_ = [("method", C.c_int), ("k", C.c_int), ("power", C.c_double), ("eps", C.c_double),
                ("fluid_mask", C.POINTER(C.c_uint8)), ("flags", C.c_uint32), ("cell_occupancy", C.c_double),
                ("r0_scale", C.c_double), ("lattice_bounds", C.c_int), ("slab_halo", C.c_double),
                ("radius", C.c_double)]


class RbfParams(C.Structure):
    _fields_ = [("k", C.c_int), ("kernel", C.c_int), ("epsilon", C.c_double), ("degree", C.c_int),
                ("smoothing", C.c_double), ("smoothing_per_point", _dp), ("fluid_mask", C.POINTER(C.c_uint8)),
                ("flags", C.c_uint32), ("chunk_planes", C.c_int)]


_i32p = C.POINTER(C.c_int32)


class LinearParams(C.Structure):
    _fields_ = [("nsimplex", C.c_int64), ("simplices", _i32p), ("neighbors", _i32p), ("transform", _dp),
                ("vertex_to_simplex", _i32p), ("min_bound", C.c_double * 3), ("max_bound", C.c_double * 3),
                ("fill_value", C.c_double), ("fluid_mask", C.POINTER(C.c_uint8)), ("flags", C.c_uint32),
                ("chunk_planes", C.c_int)]


F64 = 0
F32 = 1
FLAG_OUT_F32 = 2  # U, V, W written as float32 (main.py:230 astype, fused)
FLAG_RBF_SPD_LDS = 4  # local RBF diagnostics: SPD systems through the LDS-broadcast kernel
FLAG_RBF_PIVOTING = 8  # local RBF diagnostics: scale-invariant kernels through the pivoting solver
FLAG_KNN_REPAIR_ALL = 16  # k-NN diagnostics: near-tie repair reruns the whole launch past one tile
FLAG_SLAB_CULL_AUTO = 32  # k-NN z-slab calls: per-column cull map, cached per context and proven (ABI v10)


class DivParams(C.Structure):
    _fields_ = [("nx", C.c_int64), ("ny", C.c_int64), ("nz", C.c_int64), ("z_begin", C.c_int64),
                ("z_end", C.c_int64), ("edge_lo", C.c_int), ("edge_hi", C.c_int), ("field_dtype", C.c_int),
                ("result_dtype", C.c_int), ("dx", C.c_double), ("dy", C.c_double), ("dz", C.c_double),
                ("fluid_mask", C.POINTER(C.c_uint8))]


_u8p = C.POINTER(C.c_uint8)
MASK_BOOL = 0
MASK_BITS = 1


class MaskGrid(C.Structure):
    _fields_ = [("nx", C.c_int64), ("ny", C.c_int64), ("nz", C.c_int64), ("raw", _u8p),
                ("ax", _dp), ("ay", _dp), ("az", _dp)]


class BoundaryParams(C.Structure):
    _fields_ = [("nx", C.c_int64), ("ny", C.c_int64), ("nz", C.c_int64), ("mask", _u8p),
                ("encoding", C.c_int), ("thickness", C.c_int), ("sampling_step", C.c_int64),
                ("lo", C.c_double * 3), ("span", C.c_double * 3), ("den", C.c_double * 3)]


class FilterParams(C.Structure):
    _fields_ = [("k", C.c_int), ("threshold", C.c_double), ("mad_eps", C.c_double)]


class Stats(C.Structure):
    _fields_ = [("ms_h2d", C.c_double), ("ms_bin", C.c_double), ("ms_lattice", C.c_double), ("ms_knn", C.c_double),
                ("ms_d2h", C.c_double),
                ("ms_total", C.c_double), ("n_particles", C.c_int64), ("n_voxels", C.c_int64),
                ("n_cells", C.c_int64), ("cells", C.c_int32 * 3), ("cell_size", C.c_double * 3),
                ("r0", C.c_double), ("ms_solve", C.c_double), ("n_singular", C.c_int64),
                ("ms_stencil", C.c_double), ("n_binned", C.c_int64), ("halo_required", C.c_double),
                ("ms_cull", C.c_double), ("n_repair_tiles", C.c_int64),
                ("n_rbf_pivoted", C.c_int64)]

    def as_dict(self):
        d = {f: getattr(self, f) for f, _ in self._fields_}
        d["cells"] = list(self.cells)
        d["cell_size"] = list(self.cell_size)
        return d


EXPORTS = {
    "ptv_version": (C.c_int, []),
    "ptv_abi_sizes": (C.c_int, [C.POINTER(C.c_int64)]),
    "ptv_abi_sizes2": (C.c_int, [C.POINTER(C.c_int64)]),
    "ptv_abi_sizes3": (C.c_int, [C.POINTER(C.c_int64)]),
    "ptv_interp_linear": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(Grid), C.POINTER(LinearParams),
                                    _dp, _dp, _dp, C.POINTER(Stats)]),
    "ptv_interp_linear_dev": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(Grid),
                                        C.POINTER(LinearParams), _dp, _dp, _dp, C.c_void_p, C.POINTER(Stats)]),
    "ptv_last_error": (C.c_char_p, []),
    "ptv_device_count": (C.c_int, [C.POINTER(C.c_int)]),
    "ptv_init": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "ptv_free": (C.c_int, [C.c_void_p]),
    "ptv_interp_knn": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(Grid), C.POINTER(KnnParams),
                                 _dp, _dp, _dp, C.POINTER(Stats)]),
    "ptv_interp_knn_dev": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(Grid), C.POINTER(KnnParams),
                                     _dp, _dp, _dp, C.c_void_p, C.POINTER(Stats)]),
    "ptv_interp_rbf_local": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(Grid), C.POINTER(RbfParams),
                                       _dp, _dp, _dp, C.POINTER(Stats)]),
    "ptv_interp_rbf_local_dev": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(Grid),
                                           C.POINTER(RbfParams), _dp, _dp, _dp, C.c_void_p, C.POINTER(Stats)]),
    "ptv_divergence": (C.c_int, [C.c_void_p, C.POINTER(DivParams), C.c_void_p, C.c_void_p, C.c_void_p,
                                 C.c_void_p, C.POINTER(Stats)]),
    "ptv_divergence_dev": (C.c_int, [C.c_void_p, C.POINTER(DivParams), C.c_void_p, C.c_void_p, C.c_void_p,
                                     C.c_void_p, C.c_void_p, C.POINTER(Stats)]),
    "ptv_sample_mask": (C.c_int, [C.c_void_p, C.POINTER(MaskGrid), C.POINTER(Grid), _u8p]),
    "ptv_sample_mask_dev": (C.c_int, [C.c_void_p, C.POINTER(MaskGrid), C.POINTER(Grid), _u8p, C.c_void_p]),
    "ptv_boundary_particles": (C.c_int, [C.c_void_p, C.POINTER(BoundaryParams), _dp, _dp, _dp, C.c_int64,
                                         C.POINTER(C.c_int64)]),
    "ptv_boundary_particles_dev": (C.c_int, [C.c_void_p, C.POINTER(BoundaryParams), _dp, _dp, _dp, C.c_int64,
                                             C.POINTER(C.c_int64), C.c_void_p]),
    "ptv_filter_outliers_knn": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(FilterParams), _u8p, _dp,
                                          C.POINTER(Stats)]),
    "ptv_filter_outliers_knn_dev": (C.c_int, [C.c_void_p, C.POINTER(Particles), C.POINTER(FilterParams), _u8p,
                                              _dp, C.c_void_p, C.POINTER(Stats)]),
    "ptv_last_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "ptv_debug_stamps": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_double)]),
}

_lib = None
_lock = threading.Lock()


class PtvError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"ptv error {code}: {msg}")
        self.code = code
        self.msg = msg


def lib():
    """Load libptv_amd.so (raises if it is missing: there is no CPU fallback)."""
    global _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                raise ImportError(
                    f"{LIB_PATH} not found: build it with `python -m ptv_interpolation_amd.build` "
                    "(hipcc, gfx950). The k-NN path has no CPU fallback.")
            L = C.CDLL(LIB_PATH)
            for name, (res, args) in EXPORTS.items():
                if LIB_PATH != _DEFAULT_LIB and not hasattr(L, name):
                    continue  # an older build under PTV_LIB (same-box A/B): its missing entry points stay unbound
                fn = getattr(L, name)
                fn.restype = res
                fn.argtypes = args
            _lib = L
    return _lib


class InexactError(PtvError):
    """PTV_E_INEXACT: the slab_halo cull could not be proven exact (ptv_knn_params.slab_halo);
    ``halo_required`` is the halo that would be."""

    def __init__(self, code, msg, halo_required=None):
        super().__init__(code, msg)
        self.halo_required = halo_required


def check(rc):
    if rc != PTV_OK:
        msg = lib().ptv_last_error().decode(errors="replace")
        if rc == PTV_E_ARG:
            raise ValueError(msg)
        if rc == PTV_E_NOMEM:
            raise MemoryError(msg)
        if rc == PTV_E_UNSUPPORTED:
            raise NotImplementedError(msg)
        if rc == PTV_E_SINGULAR:
            raise np.linalg.LinAlgError(msg)
        if rc == PTV_E_INEXACT:
            raise InexactError(rc, msg)
        raise PtvError(rc, msg)
    return rc


def _check_knn(rc, st):
    if rc == PTV_E_INEXACT:
        raise InexactError(rc, lib().ptv_last_error().decode(errors="replace"), st.halo_required)
    check(rc)


def abi_sizes():
    """(C sizeof, ctypes sizeof) for each ABI struct: they must agree."""
    out = (C.c_int64 * 6)()
    check(lib().ptv_abi_sizes(out))
    py = [C.sizeof(Particles), C.sizeof(Grid), C.sizeof(KnnParams), C.sizeof(Stats), C.sizeof(RbfParams),
          C.sizeof(DivParams)]
    return list(out), py


def abi_sizes2():
    """(C sizeof, ctypes sizeof) of the pore-mask / filter structs."""
    out = (C.c_int64 * 3)()
    check(lib().ptv_abi_sizes2(out))
    return list(out), [C.sizeof(MaskGrid), C.sizeof(BoundaryParams), C.sizeof(FilterParams)]


def abi_sizes3():
    """(C sizeof, ctypes sizeof) of ptv_linear_params."""
    out = (C.c_int64 * 1)()
    check(lib().ptv_abi_sizes3(out))
    return list(out), [C.sizeof(LinearParams)]


class Triangulation:
    """The arrays of ``scipy.spatial.Delaunay(points)`` the linear kernels read, as contiguous
    int32 / float64 (``tri.transform`` is scipy's own barycentric transforms, computed on first
    access exactly as LinearNDInterpolator does).  Particles that are not vertices (Qhull
    "coplanar" points, e.g. duplicates) start their walks in the simplex Qhull assigned them."""

    def __init__(self, tri):
        self.simplices = np.ascontiguousarray(tri.simplices, dtype=np.int32)
        self.neighbors = np.ascontiguousarray(tri.neighbors, dtype=np.int32)
        self.transform = np.ascontiguousarray(tri.transform, dtype=np.float64)
        v2s = np.array(tri.vertex_to_simplex, dtype=np.int32)
        cp = np.asarray(tri.coplanar)
        if cp.size:
            v2s[cp[:, 0]] = cp[:, 1]
        self.vertex_to_simplex = np.ascontiguousarray(v2s)
        self.min_bound = [float(v) for v in tri.min_bound]
        self.max_bound = [float(v) for v in tri.max_bound]
        self.nsimplex = int(self.simplices.shape[0])

    def params(self, fill_value=0.0, fluid_mask=None, flags=0, chunk_planes=0):
        return LinearParams(self.nsimplex, self.simplices.ctypes.data_as(_i32p), self.neighbors.ctypes.data_as(_i32p),
                            as_dp(self.transform), self.vertex_to_simplex.ctypes.data_as(_i32p),
                            (C.c_double * 3)(*self.min_bound), (C.c_double * 3)(*self.max_bound), float(fill_value),
                            fluid_mask, int(flags), int(chunk_planes))


def device_count() -> int:
    n = C.c_int(0)
    check(lib().ptv_device_count(C.byref(n)))
    return n.value


def as_dp(a: np.ndarray):
    return a.ctypes.data_as(_dp)


def dev_dp(ptr: int):
    return C.cast(C.c_void_p(ptr), _dp)


class ParticleColumns:
    """The particle set as six contiguous float64 columns x, y, z, u, v, w (no copy when the
    caller's columns already are, e.g. a DataFrame's float64 block rows)."""

    def __init__(self, cols):
        cols = [np.ascontiguousarray(c, dtype=np.float64).reshape(-1) for c in cols]
        if len(cols) != 6 or len({len(c) for c in cols}) != 1:
            raise ValueError("ParticleColumns: six equal-length columns x, y, z, u, v, w")
        self.cols = cols
        self.n = len(cols[0])

    @classmethod
    def from_frame(cls, df):
        """x, y, z, u, v, w of a DataFrame coerced to float64 as interpolator.py:78-79 does."""
        return cls([df[c].to_numpy(dtype=np.float64) for c in ("x", "y", "z", "u", "v", "w")])

    @property
    def points(self):
        return np.stack(self.cols[:3], 1)

    @property
    def values(self):
        return np.stack(self.cols[3:], 1)


def _columns(points, values):
    """Six contiguous float64 columns from (N, 3) points and values, or a ParticleColumns
    passed as ``points`` (``values`` None)."""
    if isinstance(points, ParticleColumns):
        return list(points.cols)
    pts = np.ascontiguousarray(points, dtype=np.float64).reshape(-1, 3)
    vals = np.ascontiguousarray(values, dtype=np.float64).reshape(-1, 3)
    return [np.ascontiguousarray(pts[:, i]) for i in range(3)] + [np.ascontiguousarray(vals[:, i]) for i in range(3)]


def _into(out, res):
    """``res`` copied into the caller's ``out`` arrays (same contract as _outputs) when given."""
    if out is None:
        return res
    out = _outputs(out, res[0].shape, res[0].dtype)
    for o, r in zip(out, res):
        np.copyto(o, r)
    return tuple(out)


def _outputs(out, shape, dtype):
    """Three output arrays: the caller's (checked: C-contiguous, shape, dtype) or new ones."""
    if out is None:
        return [np.empty(shape, dtype=dtype) for _ in range(3)]
    out = list(out)
    for a in out:
        if a.shape != tuple(shape) or a.dtype != dtype or not a.flags.c_contiguous or not a.flags.writeable:
            raise ValueError(f"out arrays must be writeable C-contiguous {dtype} of shape {tuple(shape)}")
    return out


def _flat_tiles(gp, shape, fluid_mask, z_range):
    """A flat point list (shape (1, 1, n)) as a (npad / 64, 4, 16) point grid, padded with
    the last point: the k-NN kernels tile 4 x 4 x 4 (x, y, z) blocks of the shape, so a
    (1, 1, n) list would keep only 4 of a wave's 64 lanes busy.  Every query is independent,
    so the results are the same; returns (gp, shape, mask, unpad) or None."""
    nz, ny, nx = shape
    if nz != 1 or ny != 1 or z_range is not None or nx < 64:
        return None
    n = nx
    npad = (n + 255) // 256 * 256
    ext = [np.concatenate([a, np.full(npad - n, a[-1])]) if npad > n else a for a in gp]
    mk = None
    if fluid_mask is not None:
        m = np.ascontiguousarray(fluid_mask, dtype=np.uint8).ravel()
        mk = np.concatenate([m, np.zeros(npad - n, dtype=np.uint8)]) if npad > n else m
    return ext, (npad // 64, 4, 16), mk, (lambda a: a.reshape(-1)[:n].reshape(shape))


class Context:
    """One device context (stream + reusable device buffers)."""

    _cache = {}

    def __init__(self, device: int = 0):
        L = lib()
        h = C.c_void_p()
        check(L.ptv_init(int(device), C.byref(h)))
        self.h = h
        self.device = int(device)

    @classmethod
    def get(cls, device: int = 0) -> "Context":
        with _lock:
            ctx = cls._cache.get(device)
        if ctx is None:
            ctx = cls(device)
            with _lock:
                cls._cache[device] = ctx
        return ctx

    def close(self):
        if self.h:
            lib().ptv_free(self.h)
            self.h = None

    def last_stats(self) -> dict:
        st = Stats()
        check(lib().ptv_last_stats(self.h, C.byref(st)))
        return st.as_dict()

    def debug_stamps(self, mode=2):
        """mode 1: enable+zero, 0: disable, 2: read.  Per-wave phase cycles (mean / max)."""
        out = (C.c_double * 23)()
        check(lib().ptv_debug_stamps(self.h, int(mode), out))
        keys = ("setup", "seeds", "rows", "copy", "compute", "epilogue", "candidates", "merges", "rounds",
                "passes", "kept")
        v = list(out)
        return {"waves": v[0], "mean": dict(zip(keys, v[1:12])), "max": dict(zip(keys, v[12:23]))}

    # -- pore-mask path and outlier filter -------
    def sample_mask(self, raw, raw_axes, axes=None, grid_points=None, shape=None, z_range=None):
        """Nearest resampling of a raw byte mask (1 = value > 0.5) onto a grid -> uint8 (nz', ny, nx).

        raw: (rnz, rny, rnx) bytes; raw_axes: (x, y, z) raw voxel coordinates (host)."""
        rw = np.ascontiguousarray(raw, dtype=np.uint8)
        rnz, rny, rnx = rw.shape
        rax, ray, raz = (np.ascontiguousarray(a, dtype=np.float64).ravel() for a in raw_axes)
        M = MaskGrid(rnx, rny, rnz, rw.ctypes.data_as(_u8p), as_dp(rax), as_dp(ray), as_dp(raz))
        keep = [rw, rax, ray, raz]
        if axes is not None:
            ax, ay, az = (np.ascontiguousarray(a, dtype=np.float64).ravel() for a in axes)
            nx, ny, nz = len(ax), len(ay), len(az)
            keep += [ax, ay, az]
            G = Grid(nx, ny, nz, as_dp(ax), as_dp(ay), as_dp(az), None, None, None, 0, nz)
        else:
            nz, ny, nx = shape
            gp = [np.ascontiguousarray(a, dtype=np.float64).ravel() for a in grid_points]
            keep += gp
            G = Grid(nx, ny, nz, None, None, None, as_dp(gp[0]), as_dp(gp[1]), as_dp(gp[2]), 0, nz)
        z0, z1 = (0, nz) if z_range is None else z_range
        G.z_begin, G.z_end = z0, z1
        out = np.empty((z1 - z0, ny, nx), dtype=np.uint8)
        check(lib().ptv_sample_mask(self.h, C.byref(M), C.byref(G), out.ctypes.data_as(_u8p)))
        return out

    def boundary_particles(self, mask_bytes, encoding, thickness, step, lo, span, den):
        """Boundary voxel coordinates (x, y, z) float64 arrays; mask_bytes (nz, ny, nx) uint8."""
        mb = np.ascontiguousarray(mask_bytes, dtype=np.uint8)
        nz, ny, nx = mb.shape
        prm = BoundaryParams(nx, ny, nz, mb.ctypes.data_as(_u8p), int(encoding), int(thickness), int(step),
                             (C.c_double * 3)(*lo), (C.c_double * 3)(*span), (C.c_double * 3)(*den))
        cnt = C.c_int64(0)
        check(lib().ptv_boundary_particles(self.h, C.byref(prm), None, None, None, 0, C.byref(cnt)))
        n = cnt.value
        out = [np.empty(n, dtype=np.float64) for _ in range(3)]
        if n > 0:
            check(lib().ptv_boundary_particles(self.h, C.byref(prm), as_dp(out[0]), as_dp(out[1]),
                                               as_dp(out[2]), n, C.byref(cnt)))
        return tuple(out)

    def filter_outliers_knn(self, points, values, k=25, threshold=3.0, mad_eps=1e-6):
        """(keep uint8 (n,), kth_dist float64 (n,)) of the median/MAD k-NN filter."""
        cols = _columns(points, values)
        P = Particles(len(cols[0]), *[as_dp(c) for c in cols])
        prm = FilterParams(int(k), float(threshold), float(mad_eps))
        keep = np.empty(len(cols[0]), dtype=np.uint8)
        kth = np.empty(len(cols[0]), dtype=np.float64)
        st = Stats()
        check(lib().ptv_filter_outliers_knn(self.h, C.byref(P), C.byref(prm), keep.ctypes.data_as(_u8p),
                                            as_dp(kth), C.byref(st)))
        self.stats = st.as_dict()
        return keep, kth

    # device-pointer variants (bench.py: inputs resident in HBM)
    def sample_mask_dev(self, raw_ptr, raw_shape, raw_axes, axes_ptrs, shape, out_ptr, stream=None):
        """raw_ptr: device (rnz, rny, rnx) bytes; raw_axes: host arrays; axes_ptrs: device grid axes."""
        rnz, rny, rnx = raw_shape
        rax, ray, raz = (np.ascontiguousarray(a, dtype=np.float64).ravel() for a in raw_axes)
        M = MaskGrid(rnx, rny, rnz, C.cast(C.c_void_p(raw_ptr), _u8p), as_dp(rax), as_dp(ray), as_dp(raz))
        nz, ny, nx = shape
        G = Grid(nx, ny, nz, dev_dp(axes_ptrs[0]), dev_dp(axes_ptrs[1]), dev_dp(axes_ptrs[2]), None, None, None,
                 0, nz)
        check(lib().ptv_sample_mask_dev(self.h, C.byref(M), C.byref(G), C.cast(C.c_void_p(out_ptr), _u8p),
                                        C.c_void_p(stream) if stream else None))

    def boundary_particles_dev(self, mask_ptr, shape, thickness, step, lo, span, den, out_ptrs=None, cap=0,
                               stream=None, encoding=MASK_BOOL):
        """Returns the particle count; writes device x, y, z when out_ptrs is given and cap suffices."""
        nz, ny, nx = shape
        prm = BoundaryParams(nx, ny, nz, C.cast(C.c_void_p(mask_ptr), _u8p), int(encoding), int(thickness),
                             int(step), (C.c_double * 3)(*lo), (C.c_double * 3)(*span), (C.c_double * 3)(*den))
        cnt = C.c_int64(0)
        o = [dev_dp(p) for p in out_ptrs] if out_ptrs else [None, None, None]
        check(lib().ptv_boundary_particles_dev(self.h, C.byref(prm), o[0], o[1], o[2], int(cap), C.byref(cnt),
                                               C.c_void_p(stream) if stream else None))
        return cnt.value

    def filter_outliers_knn_dev(self, n, col_ptrs, keep_ptr, kth_ptr, k=25, threshold=3.0, mad_eps=1e-6,
                                stream=None):
        """col_ptrs: six device float64 columns x, y, z, u, v, w."""
        P = Particles(int(n), *[dev_dp(p) for p in col_ptrs])
        prm = FilterParams(int(k), float(threshold), float(mad_eps))
        st = Stats()
        check(lib().ptv_filter_outliers_knn_dev(self.h, C.byref(P), C.byref(prm),
                                                C.cast(C.c_void_p(keep_ptr), _u8p),
                                                dev_dp(kth_ptr) if kth_ptr else None,
                                                C.c_void_p(stream) if stream else None, C.byref(st)))
        return st.as_dict()

    # -- host buffers ------------------------------------------------------
    def interp_knn(self, points, values, axes=None, grid_points=None, shape=None, method=METHOD_IDW, k=8,
                   power=2.0, eps=1e-10, fluid_mask=None, flags=0, z_range=None, cell_occupancy=0.0,
                   r0_scale=0.0, lattice_bounds=0, slab_halo=0.0, out=None, radius=0.0):
        """Host-array k-NN interpolation. Returns (U, V, W) float64 (nz', ny, nx).

        ``out``: optional three C-contiguous (nz', ny, nx) arrays of the output dtype (e.g.
        z-slices of the caller's full arrays) written in place by the D2H."""
        cols = _columns(points, values)
        P = Particles(len(cols[0]), *[as_dp(c) for c in cols])
        keep = list(cols)
        if axes is not None:
            ax, ay, az = (np.ascontiguousarray(a, dtype=np.float64).ravel() for a in axes)
            nx, ny, nz = len(ax), len(ay), len(az)
            keep += [ax, ay, az]
            G = Grid(nx, ny, nz, as_dp(ax), as_dp(ay), as_dp(az), None, None, None, 0, nz)
        else:
            gp = [np.ascontiguousarray(a, dtype=np.float64).ravel() for a in grid_points]
            ft = _flat_tiles(gp, shape, fluid_mask, z_range)
            if ft is not None:
                gp, tshape, fm, unpad = ft
                res = self.interp_knn(points, values, grid_points=gp, shape=tshape, method=method, k=k,
                                      power=power, eps=eps, fluid_mask=fm, flags=flags,
                                      cell_occupancy=cell_occupancy, r0_scale=r0_scale,
                                      lattice_bounds=lattice_bounds, slab_halo=slab_halo, radius=radius)
                return _into(out, tuple(unpad(a) for a in res))
            nz, ny, nx = shape
            keep += gp
            G = Grid(nx, ny, nz, None, None, None, as_dp(gp[0]), as_dp(gp[1]), as_dp(gp[2]), 0, nz)
        z0, z1 = (0, nz) if z_range is None else z_range
        G.z_begin, G.z_end = z0, z1
        mk = None
        if fluid_mask is not None:
            mk = np.ascontiguousarray(fluid_mask, dtype=np.uint8).reshape(nz, ny, nx)
            keep.append(mk)
        prm = KnnParams(method, int(k), float(power), float(eps),
                        mk.ctypes.data_as(C.POINTER(C.c_uint8)) if mk is not None else None, flags,
                        float(cell_occupancy), float(r0_scale), int(lattice_bounds), float(slab_halo),
                        float(radius))
        odt = np.float32 if flags & FLAG_OUT_F32 else np.float64
        out = _outputs(out, (z1 - z0, ny, nx), odt)
        st = Stats()
        rc = lib().ptv_interp_knn(self.h, C.byref(P), C.byref(G), C.byref(prm),
                                  as_dp(out[0]), as_dp(out[1]), as_dp(out[2]), C.byref(st))
        self.stats = st.as_dict()
        _check_knn(rc, st)
        return tuple(out)

    def interp_rbf(self, points, values, axes=None, grid_points=None, shape=None, k=20,
                   kernel="thin_plate_spline", epsilon=1.0, degree=1, smoothing=0.0, fluid_mask=None, flags=0,
                   z_range=None, chunk_planes=0, out=None):
        """Host-array local RBF (scipy RBFInterpolator(neighbors=k) semantics; the arguments are
        already resolved by ptv_interpolation_amd.rbf).  ``smoothing``: scalar or (n,) array.
        Returns (U, V, W) float64 (nz', ny, nx)."""
        cols = _columns(points, values)
        P = Particles(len(cols[0]), *[as_dp(c) for c in cols])
        keep = list(cols)
        if axes is not None:
            ax, ay, az = (np.ascontiguousarray(a, dtype=np.float64).ravel() for a in axes)
            nx, ny, nz = len(ax), len(ay), len(az)
            keep += [ax, ay, az]
            G = Grid(nx, ny, nz, as_dp(ax), as_dp(ay), as_dp(az), None, None, None, 0, nz)
        else:
            gp = [np.ascontiguousarray(a, dtype=np.float64).ravel() for a in grid_points]
            ft = _flat_tiles(gp, shape, fluid_mask, z_range)
            if ft is not None:
                gp, tshape, fm, unpad = ft
                res = self.interp_rbf(points, values, grid_points=gp, shape=tshape, k=k, kernel=kernel,
                                      epsilon=epsilon, degree=degree, smoothing=smoothing, fluid_mask=fm,
                                      flags=flags, chunk_planes=chunk_planes)
                return _into(out, tuple(unpad(a) for a in res))
            nz, ny, nx = shape
            keep += gp
            G = Grid(nx, ny, nz, None, None, None, as_dp(gp[0]), as_dp(gp[1]), as_dp(gp[2]), 0, nz)
        z0, z1 = (0, nz) if z_range is None else z_range
        G.z_begin, G.z_end = z0, z1
        mk = None
        if fluid_mask is not None:
            mk = np.ascontiguousarray(fluid_mask, dtype=np.uint8).reshape(nz, ny, nx)
            keep.append(mk)
        sm_arr = None
        if np.ndim(smoothing) > 0:
            sm_arr = np.ascontiguousarray(smoothing, dtype=np.float64).ravel()
            keep.append(sm_arr)
        prm = RbfParams(int(k), RBF_KERNELS[kernel], float(epsilon), int(degree),
                        0.0 if sm_arr is not None else float(smoothing),
                        as_dp(sm_arr) if sm_arr is not None else None,
                        mk.ctypes.data_as(C.POINTER(C.c_uint8)) if mk is not None else None, int(flags),
                        int(chunk_planes))
        out = _outputs(out, (z1 - z0, ny, nx), np.float64)
        st = Stats()
        check(lib().ptv_interp_rbf_local(self.h, C.byref(P), C.byref(G), C.byref(prm),
                                         as_dp(out[0]), as_dp(out[1]), as_dp(out[2]), C.byref(st)))
        self.stats = st.as_dict()
        return tuple(out)

    def interp_linear(self, points, values, tri, axes=None, grid_points=None, shape=None, fill_value=0.0,
                      fluid_mask=None, flags=0, z_range=None, chunk_planes=0, out=None):
        """Host-array linear (Delaunay) interpolation (griddata(method='linear') semantics) over
        ``tri`` (a Triangulation of these points).  Returns (U, V, W) float64 (nz', ny, nx)."""
        cols = _columns(points, values)
        P = Particles(len(cols[0]), *[as_dp(c) for c in cols])
        keep = list(cols)
        if axes is not None:
            ax, ay, az = (np.ascontiguousarray(a, dtype=np.float64).ravel() for a in axes)
            nx, ny, nz = len(ax), len(ay), len(az)
            keep += [ax, ay, az]
            G = Grid(nx, ny, nz, as_dp(ax), as_dp(ay), as_dp(az), None, None, None, 0, nz)
        else:
            gp = [np.ascontiguousarray(a, dtype=np.float64).ravel() for a in grid_points]
            ft = _flat_tiles(gp, shape, fluid_mask, z_range)
            if ft is not None:
                gp, tshape, fm, unpad = ft
                res = self.interp_linear(points, values, tri, grid_points=gp, shape=tshape, fill_value=fill_value,
                                         fluid_mask=fm, flags=flags, chunk_planes=chunk_planes)
                return _into(out, tuple(unpad(a) for a in res))
            nz, ny, nx = shape
            keep += gp
            G = Grid(nx, ny, nz, None, None, None, as_dp(gp[0]), as_dp(gp[1]), as_dp(gp[2]), 0, nz)
        z0, z1 = (0, nz) if z_range is None else z_range
        G.z_begin, G.z_end = z0, z1
        mk = None
        if fluid_mask is not None:
            mk = np.ascontiguousarray(fluid_mask, dtype=np.uint8).reshape(nz, ny, nx)
            keep.append(mk)
        prm = tri.params(fill_value, mk.ctypes.data_as(C.POINTER(C.c_uint8)) if mk is not None else None, flags,
                         chunk_planes)
        out = _outputs(out, (z1 - z0, ny, nx), np.float64)
        st = Stats()
        check(lib().ptv_interp_linear(self.h, C.byref(P), C.byref(G), C.byref(prm),
                                      as_dp(out[0]), as_dp(out[1]), as_dp(out[2]), C.byref(st)))
        self.stats = st.as_dict()
        return tuple(out)

    def interp_linear_dev(self, n, pptrs, nx, ny, nz, tri_ptrs, nsimplex, min_bound, max_bound, axes_ptrs=None,
                          point_ptrs=None, out_ptrs=None, fill_value=0.0, mask_ptr=0, flags=0, z_range=None,
                          stream=0, chunk_planes=0):
        """Device-pointer linear interpolation; tri_ptrs: device (simplices, neighbors, transform,
        vertex_to_simplex).  Returns the call's stats."""
        P = Particles(int(n), *[dev_dp(p) for p in pptrs])
        if axes_ptrs is not None:
            G = Grid(nx, ny, nz, *[dev_dp(p) for p in axes_ptrs], None, None, None, 0, nz)
        else:
            G = Grid(nx, ny, nz, None, None, None, *[dev_dp(p) for p in point_ptrs], 0, nz)
        z0, z1 = (0, nz) if z_range is None else z_range
        G.z_begin, G.z_end = z0, z1
        i32 = lambda p: C.cast(C.c_void_p(p), _i32p)
        prm = LinearParams(int(nsimplex), i32(tri_ptrs[0]), i32(tri_ptrs[1]), dev_dp(tri_ptrs[2]), i32(tri_ptrs[3]),
                           (C.c_double * 3)(*min_bound), (C.c_double * 3)(*max_bound), float(fill_value),
                           C.cast(C.c_void_p(mask_ptr), C.POINTER(C.c_uint8)) if mask_ptr else None, int(flags),
                           int(chunk_planes))
        st = Stats()
        check(lib().ptv_interp_linear_dev(self.h, C.byref(P), C.byref(G), C.byref(prm),
                                          *[dev_dp(p) for p in out_ptrs], C.c_void_p(stream) if stream else None,
                                          C.byref(st)))
        return st.as_dict()

    def interp_rbf_dev(self, n, pptrs, nx, ny, nz, axes_ptrs=None, point_ptrs=None, out_ptrs=None, k=20,
                       kernel="thin_plate_spline", epsilon=1.0, degree=1, smoothing=0.0, smoothing_ptr=0,
                       mask_ptr=0, flags=0, z_range=None, stream=0, chunk_planes=0):
        """Device-pointer local RBF (inputs resident in HBM); returns the call's stats."""
        P = Particles(int(n), *[dev_dp(p) for p in pptrs])
        if axes_ptrs is not None:
            G = Grid(nx, ny, nz, *[dev_dp(p) for p in axes_ptrs], None, None, None, 0, nz)
        else:
            G = Grid(nx, ny, nz, None, None, None, *[dev_dp(p) for p in point_ptrs], 0, nz)
        z0, z1 = (0, nz) if z_range is None else z_range
        G.z_begin, G.z_end = z0, z1
        prm = RbfParams(int(k), RBF_KERNELS[kernel], float(epsilon), int(degree), float(smoothing),
                        dev_dp(smoothing_ptr) if smoothing_ptr else None,
                        C.cast(C.c_void_p(mask_ptr), C.POINTER(C.c_uint8)) if mask_ptr else None, int(flags),
                        int(chunk_planes))
        st = Stats()
        check(lib().ptv_interp_rbf_local_dev(self.h, C.byref(P), C.byref(G), C.byref(prm),
                                             *[dev_dp(p) for p in out_ptrs], C.c_void_p(stream or 0),
                                             C.byref(st)))
        return st.as_dict()

    # -- device buffers (integer device pointers, e.g. torch tensor data_ptr()) --
    def interp_knn_dev(self, n, pptrs, nx, ny, nz, axes_ptrs=None, point_ptrs=None, out_ptrs=None,
                       method=METHOD_IDW, k=8, power=2.0, eps=1e-10, mask_ptr=0, flags=0, z_range=None,
                       stream=0, cell_occupancy=0.0, r0_scale=0.0, lattice_bounds=0, slab_halo=0.0, radius=0.0):
        """Device-pointer k-NN interpolation (inputs resident in HBM), enqueued on `stream`;
        returns the call's stats.  ``slab_halo`` > 0: see ptv_knn_params.slab_halo (raises
        InexactError carrying ``halo_required`` when the halo is too small)."""
        P = Particles(int(n), *[dev_dp(p) for p in pptrs])
        if axes_ptrs is not None:
            G = Grid(nx, ny, nz, *[dev_dp(p) for p in axes_ptrs], None, None, None, 0, nz)
        else:
            G = Grid(nx, ny, nz, None, None, None, *[dev_dp(p) for p in point_ptrs], 0, nz)
        z0, z1 = (0, nz) if z_range is None else z_range
        G.z_begin, G.z_end = z0, z1
        prm = KnnParams(method, int(k), float(power), float(eps),
                        C.cast(C.c_void_p(mask_ptr), C.POINTER(C.c_uint8)) if mask_ptr else None, flags,
                        float(cell_occupancy), float(r0_scale), int(lattice_bounds), float(slab_halo),
                        float(radius))
        st = Stats()
        rc = lib().ptv_interp_knn_dev(self.h, C.byref(P), C.byref(G), C.byref(prm),
                                      *[dev_dp(p) for p in out_ptrs], C.c_void_p(stream or 0), C.byref(st))
        _check_knn(rc, st)
        return st.as_dict()

    # -- consistent divergence (physics.py:6-53) ---------------------------
    def divergence(self, u, v, w, fluid_mask, dx, dy, dz, result_dtype=None, z_range=None, edges=(True, True)):
        """Host-array divergence of (nz, ny, nx) fields; returns (z1 - z0, ny, nx) of
        ``result_dtype`` (default: the fields' dtype).  ``edges``: whether buffer plane 0 /
        nz-1 is a domain edge (else a halo plane, read but not computed)."""
        ft = np.result_type(u.dtype, v.dtype, w.dtype)
        if ft not in (np.float32, np.float64):
            ft = np.dtype(np.float64)
        rt = np.dtype(result_dtype) if result_dtype is not None else np.dtype(ft)
        f = [np.ascontiguousarray(a, dtype=ft) for a in (u, v, w)]
        nz, ny, nx = f[0].shape
        mk = np.ascontiguousarray(fluid_mask, dtype=bool).view(np.uint8).reshape(nz, ny, nx)
        z0, z1 = (0, nz) if z_range is None else z_range
        prm = DivParams(nx, ny, nz, z0, z1, int(bool(edges[0])), int(bool(edges[1])),
                        F32 if ft == np.float32 else F64, F32 if rt == np.float32 else F64,
                        float(dx), float(dy), float(dz), mk.ctypes.data_as(C.POINTER(C.c_uint8)))
        out = np.empty((z1 - z0, ny, nx), dtype=rt)
        st = Stats()
        check(lib().ptv_divergence(self.h, C.byref(prm), *[a.ctypes.data_as(C.c_void_p) for a in f],
                                   out.ctypes.data_as(C.c_void_p), C.byref(st)))
        self.stats = st.as_dict()
        return out

    def divergence_dev(self, nx, ny, nz, ptrs, mask_ptr, out_ptr, dx, dy, dz, field_dtype=F64, result_dtype=F64,
                       z_range=None, edges=(True, True), stream=0):
        """Device-pointer divergence (fields, mask and output resident in HBM); returns stats."""
        z0, z1 = (0, nz) if z_range is None else z_range
        prm = DivParams(nx, ny, nz, z0, z1, int(bool(edges[0])), int(bool(edges[1])), int(field_dtype),
                        int(result_dtype), float(dx), float(dy), float(dz),
                        C.cast(C.c_void_p(mask_ptr), C.POINTER(C.c_uint8)) if mask_ptr else None)
        st = Stats()
        check(lib().ptv_divergence_dev(self.h, C.byref(prm), *[C.c_void_p(p) for p in ptrs], C.c_void_p(out_ptr),
                                       C.c_void_p(stream or 0), C.byref(st)))
        return st.as_dict()
