"""raytracing-programs_amd — Python host bindings of the MI355X raycaster.

The product is C: ``lib/libraycast_hip.so`` (HIP kernels + the C-ABI declared in
``include/raycast_hip.h``) and ``lib/libraycast_front.so`` (scene parser / P3 writer with the
reference's names and behaviour, C/parse.c, C/objects.c, C/ppm.c).  This module only binds
them with ctypes so tests and ``bench.py`` can drive the same entry points the C CLI uses:

    scene = Scene.from_file("tests/golden/scenes/quadric.scene")   # parse_json (C/parse.c:13)
    img = render(scene, 4096, 4096, depth=6, mode="parity")       # raycast (C/raycast.h:8)

There is no CPU fallback: loading fails loudly if the shared libraries are missing, and a
render fails if no GPU is present.  Import name: ``raytracing_programs_amd`` (the directory
name has a hyphen; ``__graft_entry__`` and tests load it by path).
"""
import ctypes
import os
import sys
import threading

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_DIR = os.path.join(PKG_DIR, "lib")
BIN_DIR = os.path.join(PKG_DIR, "bin")
ROOT_DIR = os.path.dirname(PKG_DIR)

MODE_PARITY = 0
MODE_FAST = 1
MODE_CUDA = 2   # the CUDA port's semantics (include/raycast_hip.h RC_MODE_CUDA)
MODES = {"parity": MODE_PARITY, "fast": MODE_FAST, "cuda": MODE_CUDA}


# ------------------------------------------------------------------ ABI structs --
class ShapeT(ctypes.Structure):
    """shape_t, C/objects.h:15-49 (104 bytes)."""
    _fields_ = [("diffuse_color", ctypes.c_float * 3), ("specular_color", ctypes.c_float * 3),
                ("position", ctypes.c_float * 3), ("reflectivity", ctypes.c_float),
                ("refractivity", ctypes.c_float), ("ior", ctypes.c_float),
                ("u", ctypes.c_float * 10), ("type", ctypes.c_int),
                ("next", ctypes.c_void_p)]


class LightT(ctypes.Structure):
    """light_t, C/objects.h:51-61 (72 bytes)."""
    _fields_ = [("position", ctypes.c_float * 3), ("color", ctypes.c_float * 3),
                ("radial_coef", ctypes.c_float * 3), ("theta", ctypes.c_float),
                ("cos_theta", ctypes.c_float), ("a0", ctypes.c_float),
                ("direction", ctypes.c_float * 3), ("type", ctypes.c_int),
                ("next", ctypes.c_void_p)]


class JsonDataT(ctypes.Structure):
    """json_data_t, C/parse.h:11-18."""
    _fields_ = [("camera_width", ctypes.c_float), ("camera_height", ctypes.c_float),
                ("shapes_list", ctypes.POINTER(ShapeT)), ("lights_list", ctypes.POINTER(LightT)),
                ("num_shapes", ctypes.c_int), ("num_lights", ctypes.c_int)]


class PPMFormat(ctypes.Structure):
    """PPMFormat, C/ppm.h:6-12."""
    _fields_ = [("width", ctypes.c_int), ("height", ctypes.c_int), ("size", ctypes.c_int),
                ("maxColor", ctypes.c_uint8), ("depth", ctypes.c_uint8),
                ("tupleType", ctypes.c_char_p), ("pixmap", ctypes.c_void_p)]


class RcOptions(ctypes.Structure):
    _fields_ = [("max_recursion", ctypes.c_int), ("mode", ctypes.c_int),
                ("num_gpus", ctypes.c_int), ("device", ctypes.c_int)]


class RcTiming(ctypes.Structure):
    _fields_ = [("total_ms", ctypes.c_double), ("kernel_ms", ctypes.c_double),
                ("resolve_ms", ctypes.c_double), ("d2h_ms", ctypes.c_double),
                ("dep_pixels", ctypes.c_int64), ("zero_normalize", ctypes.c_int64),
                ("frames_checked", ctypes.c_int64), ("frames_failed", ctypes.c_int64)]


class RcPhaseStats(ctypes.Structure):
    _fields_ = [("calls", ctypes.c_int), ("parity", ctypes.c_int), ("phase_a_ms", ctypes.c_double),
                ("compact_ms", ctypes.c_double), ("resolve_ms", ctypes.c_double),
                ("phase_c_ms", ctypes.c_double), ("render_ms", ctypes.c_double),
                ("total_ms", ctypes.c_double)]


class RcShardStats(ctypes.Structure):
    _fields_ = [("ranks", ctypes.c_int), ("total_ms", ctypes.c_double),
                ("device_ms", ctypes.c_double), ("local_ms", ctypes.c_double),
                ("exchange_in_ms", ctypes.c_double), ("resolve_ms", ctypes.c_double),
                ("phase_c_ms", ctypes.c_double), ("image_ms", ctypes.c_double),
                ("dep_pixels", ctypes.c_int64), ("zero_normalize", ctypes.c_int64),
                ("entry_bytes", ctypes.c_int64), ("carry_bytes", ctypes.c_int64),
                ("image_bytes", ctypes.c_int64)]


class RcRankStats(ctypes.Structure):
    _fields_ = [("rank", ctypes.c_int), ("rows", ctypes.c_int), ("local_ms", ctypes.c_double),
                ("exchange_ms", ctypes.c_double), ("total_ms", ctypes.c_double),
                ("dep_pixels", ctypes.c_int64)]


class RcResolverStats(ctypes.Structure):
    _fields_ = [("frames", ctypes.c_int64), ("resolve_ms_min", ctypes.c_double),
                ("resolve_ms_max", ctypes.c_double), ("resolve_ms_mean", ctypes.c_double),
                ("grid", ctypes.c_int32), ("res_cus", ctypes.c_int32),
                ("wg_per_cu", ctypes.c_int32), ("wg_per_cu_max", ctypes.c_int32),
                ("regs", ctypes.c_int32), ("scratch_bytes", ctypes.c_int32),
                ("lds_bytes", ctypes.c_int32), ("team_blocks", ctypes.c_int32),
                ("scan_rounds_max", ctypes.c_int32), ("cscan_rounds_max", ctypes.c_int32),
                ("resolve_rounds_max", ctypes.c_int32), ("pad", ctypes.c_int32),
                ("spin_wait_us_max", ctypes.c_double * 4),
                ("clock_mhz_min", ctypes.c_int32), ("clock_mhz_max", ctypes.c_int32)]


TUNING_FIELDS = ["side", "split_shade", "resolve_shared", "resolve_lds_kb", "resolve_grid",
                 "team_blocks", "helpers", "hand_run", "long_len", "wave_k", "resolve_k", "coop",
                 "dep_fast", "o0", "phase_c_finish", "single_res_cus", "pipe_res_cus",
                 "pipe_resolvers", "pipe_slots", "pipe_timing", "pipe_slotstreams", "overlap_d2h",
                 "staged_d2h", "prefault", "copy_threads", "side_blocks", "comp_stream",
                 "block_min", "pipe_inres", "x0", "resolve_clean",
                 "shard_lone", "team_cscan", "pipe_order", "pipe_helpers", "patch_host",
                 "share_device", "headb_first", "pipe_last_whole"]


class RcTuning(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in TUNING_FIELDS]


assert ctypes.sizeof(ShapeT) == 104 and ctypes.sizeof(LightT) == 72

# the functions include/raycast_hip.h declares, per library
HIP_EXPORTS = ["raycast", "rc_default_options", "rc_scene_create", "rc_scene_destroy",
               "rc_scene_parity_defined", "rc_render", "rc_render_device", "rc_last_kernel_ms",
               "rc_profile_begin", "rc_profile_end", "rc_version", "rc_frame_submit",
               "rc_frames_wait", "rc_pipe_reset", "rc_group_unique_id", "rc_group_create_rank",
               "rc_group_create_local", "rc_group_destroy", "rc_group_size",
               "rc_group_transport", "rc_render_sharded", "rc_group_last_stats",
               "rc_default_tuning", "rc_set_tuning", "rc_get_tuning", "rc_lone_frames_check",
               "rc_debug_inject_error", "rc_group_debug_bound", "rc_resolver_stats_get",
               "rc_group_rank_stats", "rc_debug_scatter_selftest"]
FRONT_EXPORTS = ["add_new_sphere", "add_new_plane", "add_new_quadric", "free_shape_list",
                 "free_light_list", "add_new_spot_light", "add_new_point_light", "parse_json",
                 "set_to_black", "ppm_WriteOutP3", "ppm_clamp"]

_libs = {}


def _load(name):
    if name not in _libs:
        path = os.path.join(LIB_DIR, name)
        if not os.path.exists(path):
            raise RuntimeError(f"{path} is missing: build with `make` (or __graft_entry__.build())")
        _libs[name] = ctypes.CDLL(path, mode=ctypes.RTLD_GLOBAL)
    return _libs[name]


def front_lib():
    lib = _load("libraycast_front.so")
    lib.parse_json.argtypes = [ctypes.c_void_p, ctypes.POINTER(JsonDataT)]
    lib.parse_json.restype = None
    lib.free_shape_list.argtypes = [ctypes.c_void_p]
    lib.free_shape_list.restype = ctypes.c_void_p
    lib.free_light_list.argtypes = [ctypes.c_void_p]
    lib.free_light_list.restype = ctypes.c_void_p
    lib.ppm_WriteOutP3.argtypes = [PPMFormat, ctypes.c_void_p]
    lib.ppm_WriteOutP3.restype = None
    return lib


_torch_tried = False


def _one_hip_runtime():
    """PyTorch-ROCm bundles its own HIP runtime (torch/lib/libamdhip64.so, SONAME
    libamdhip64.so.7, which torch's libraries reference as plain `libamdhip64.so`).  If
    libraycast_hip.so loaded /opt/rocm's runtime first and torch were imported later, the
    loader would map a second HIP runtime into the process (two device contexts; their
    teardown corrupts the heap at exit).  Importing torch first makes libraycast_hip.so's
    `libamdhip64.so.7` / `librccl.so.1` resolve to the runtime already loaded: one per
    process.  Without torch, /opt/rocm's runtime is the only one."""
    global _torch_tried
    if _torch_tried or "torch" in sys.modules:
        return
    _torch_tried = True   # once: a failed import is not retried on every call
    try:
        import torch  # noqa: F401
    except ImportError:
        pass


_HIP_LOCK = threading.Lock()
_hip = None


def hip_lib():
    # RC_HIP_LIB selects a diagnostic build (e.g. libraycast_hip_stamps.so); never the default.
    # Under a lock: threads making their first call at once must not load the library while
    # another is still importing torch (a half-imported torch is already in sys.modules, and
    # the library would then map /opt/rocm's HIP runtime beside torch's: _one_hip_runtime).
    # Once bound, later calls take the cached handle without the lock.
    lib = _hip
    if lib is not None:
        return lib
    with _HIP_LOCK:
        return _hip_lib_locked()


def _hip_lib_locked():
    global _hip
    if _hip is not None:
        return _hip
    _one_hip_runtime()
    lib = _load(os.environ.get("RC_HIP_LIB", "libraycast_hip.so"))
    lib.rc_scene_create.argtypes = [ctypes.POINTER(JsonDataT)]
    lib.rc_scene_create.restype = ctypes.c_void_p
    lib.rc_scene_destroy.argtypes = [ctypes.c_void_p]
    lib.rc_scene_parity_defined.argtypes = [ctypes.c_void_p]
    lib.rc_render.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                              ctypes.POINTER(RcOptions), ctypes.c_void_p, ctypes.POINTER(RcTiming)]
    lib.rc_render_device.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                     ctypes.c_int, ctypes.c_int, ctypes.POINTER(RcOptions),
                                     ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(RcTiming)]
    lib.rc_frame_submit.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                    ctypes.POINTER(RcOptions), ctypes.c_void_p]
    lib.rc_frames_wait.argtypes = [ctypes.POINTER(RcTiming)]
    lib.rc_pipe_reset.argtypes = []
    lib.rc_last_kernel_ms.restype = ctypes.c_double
    lib.rc_version.restype = ctypes.c_char_p
    lib.rc_default_options.argtypes = [ctypes.POINTER(RcOptions), ctypes.c_int]
    lib.rc_profile_end.argtypes = [ctypes.POINTER(RcPhaseStats)]
    lib.rc_group_unique_id.argtypes = [ctypes.c_char_p]
    lib.rc_group_create_rank.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_char_p, ctypes.c_int]
    lib.rc_group_create_rank.restype = ctypes.c_void_p
    lib.rc_group_create_local.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.c_int]
    lib.rc_group_create_local.restype = ctypes.c_void_p
    lib.rc_group_destroy.argtypes = [ctypes.c_void_p]
    lib.rc_group_size.argtypes = [ctypes.c_void_p]
    lib.rc_group_transport.argtypes = [ctypes.c_void_p]
    lib.rc_render_sharded.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int, ctypes.c_int,
                                      ctypes.POINTER(RcOptions), ctypes.c_void_p,
                                      ctypes.POINTER(RcTiming)]
    lib.rc_group_last_stats.argtypes = [ctypes.c_void_p, ctypes.POINTER(RcShardStats)]
    lib.rc_group_debug_bound.argtypes = [ctypes.c_void_p, ctypes.c_longlong]
    lib.rc_default_tuning.argtypes = [ctypes.POINTER(RcTuning)]
    lib.rc_default_tuning.restype = None
    lib.rc_get_tuning.argtypes = [ctypes.POINTER(RcTuning)]
    lib.rc_get_tuning.restype = None
    lib.rc_set_tuning.argtypes = [ctypes.POINTER(RcTuning)]
    lib.rc_lone_frames_check.argtypes = [ctypes.POINTER(ctypes.c_int64),
                                         ctypes.POINTER(ctypes.c_int64)]
    lib.rc_debug_inject_error.argtypes = [ctypes.c_int]
    lib.rc_resolver_stats_get.argtypes = [ctypes.c_int, ctypes.POINTER(RcResolverStats)]
    lib.rc_group_rank_stats.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.POINTER(RcRankStats)]
    _hip = lib
    return lib


_libc = ctypes.CDLL(None)
_libc.fopen.restype = ctypes.c_void_p
_libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
_libc.fclose.argtypes = [ctypes.c_void_p]
_libc.open_memstream.restype = ctypes.c_void_p
_libc.open_memstream.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_size_t)]
_libc.free.argtypes = [ctypes.c_void_p]


_PACK_LOCK = threading.Lock()


class Scene:
    """A parsed scene: the reference's json_data_t lists plus the packed device scene."""

    def __init__(self, js):
        self.js = js
        self._packed = None

    @classmethod
    def from_file(cls, path):
        """parse_json (C/parse.c:13) through libraycast_front.so.  Like the reference, a
        malformed file makes the parser print to stderr and exit(1)."""
        lib = front_lib()
        f = _libc.fopen(os.fsencode(path), b"r")
        if not f:
            raise FileNotFoundError(path)
        js = JsonDataT()
        try:
            lib.parse_json(f, ctypes.byref(js))
        finally:
            _libc.fclose(f)
        return cls(js)

    @property
    def num_shapes(self):
        return self.js.num_shapes

    @property
    def num_lights(self):
        return self.js.num_lights

    def shapes(self):
        out, p = [], self.js.shapes_list
        while p:
            out.append(p.contents)
            p = ctypes.cast(p.contents.next, ctypes.POINTER(ShapeT))
        return out

    def lights(self):
        out, p = [], self.js.lights_list
        while p:
            out.append(p.contents)
            p = ctypes.cast(p.contents.next, ctypes.POINTER(LightT))
        return out

    def packed(self):
        """rc_scene handle (packed image + phantom record) for the HIP library."""
        with _PACK_LOCK:   # render threads sharing a Scene create its handle once
            if self._packed is None:
                h = hip_lib().rc_scene_create(ctypes.byref(self.js))
                if not h:
                    raise RuntimeError("rc_scene_create failed")
                self._packed = h
            return self._packed

    def parity_defined(self):
        return bool(hip_lib().rc_scene_parity_defined(self.packed()))

    def close(self):
        if self._packed is not None:
            hip_lib().rc_scene_destroy(self._packed)
            self._packed = None
        lib = front_lib()
        if self.js.shapes_list:
            lib.free_shape_list(ctypes.cast(self.js.shapes_list, ctypes.c_void_p))
            self.js.shapes_list = None
        if self.js.lights_list:
            lib.free_light_list(ctypes.cast(self.js.lights_list, ctypes.c_void_p))
            self.js.lights_list = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def get_tuning(default=False):
    """The process-wide schedule tuning (rc_get_tuning / rc_default_tuning) as a dict."""
    t = RcTuning()
    (hip_lib().rc_default_tuning if default else hip_lib().rc_get_tuning)(ctypes.byref(t))
    return {n: getattr(t, n) for n in TUNING_FIELDS}


def set_tuning(**fields):
    """Change tuning fields (the rest keep their current values); rc_set_tuning validates."""
    cur = get_tuning()
    unknown = set(fields) - set(cur)
    if unknown:
        raise KeyError(f"unknown tuning fields {sorted(unknown)}")
    cur.update(fields)
    t = RcTuning(**cur)
    if hip_lib().rc_set_tuning(ctypes.byref(t)) != 0:
        raise ValueError(f"rc_set_tuning rejected {fields}")


class tuned:
    """Context manager: `with tuned(side=0): ...` renders with the given tuning, then restores."""

    def __init__(self, **fields):
        self.fields = fields

    def __enter__(self):
        self.saved = get_tuning()
        set_tuning(**self.fields)
        return self

    def __exit__(self, *exc):
        set_tuning(**self.saved)
        return False


def options(depth=6, mode="parity", gpus=1, device=0):
    opt = RcOptions()
    opt.max_recursion = depth + 1
    opt.mode = MODES[mode] if isinstance(mode, str) else int(mode)
    opt.num_gpus = gpus
    opt.device = device
    return opt


def render(scene, width, height, depth=6, mode="parity", gpus=1, device=0, timing=None, out=None):
    """Render to a host array [H, W, 3] uint8 through rc_render (the raycast() path); `out`
    (optional) is the caller's C-contiguous pixmap, like the reference's malloc'd one."""
    lib = hip_lib()
    if out is None:
        out = np.empty((height, width, 3), dtype=np.uint8)
    assert out.shape == (height, width, 3) and out.dtype == np.uint8 and out.flags.c_contiguous
    t = RcTiming()
    opt = options(depth, mode, gpus, device)
    rc = lib.rc_render(scene.packed(), width, height, ctypes.byref(opt),
                       out.ctypes.data_as(ctypes.c_void_p), ctypes.byref(t))
    if rc != 0:
        raise RuntimeError("rc_render failed (no GPU, or HIP error: see stderr)")
    if timing is not None:
        timing.update({k: getattr(t, k) for k, _ in RcTiming._fields_})
    return out


def render_device(scene, width, height, d_out_ptr, stream_ptr=None, depth=6, mode="parity",
                  row0=0, row_step=1, nrows=None, timing=None):
    """Render rows row0, row0+row_step, ... into device memory at d_out_ptr (nrows*W*3 B)."""
    lib = hip_lib()
    nrows = height if nrows is None else nrows
    opt = options(depth, mode)
    t = RcTiming()
    rc = lib.rc_render_device(scene.packed(), width, height, row0, row_step, nrows,
                              ctypes.byref(opt), ctypes.c_void_p(d_out_ptr),
                              ctypes.c_void_p(stream_ptr or 0),
                              ctypes.byref(t) if timing is not None else None)
    if rc != 0:
        raise RuntimeError("rc_render_device failed (see stderr)")
    if timing is not None:
        timing.update({k: getattr(t, k) for k, _ in RcTiming._fields_})


def frame_submit(scene, width, height, d_out_ptr, depth=6, mode="parity"):
    """Enqueue one whole image into device memory at d_out_ptr (W*H*3 B) with frames in
    flight (rc_frame_submit); returns at once.  Pair with frames_wait()."""
    opt = options(depth, mode)
    if hip_lib().rc_frame_submit(scene.packed(), width, height, ctypes.byref(opt),
                                 ctypes.c_void_p(d_out_ptr)) != 0:
        raise RuntimeError("rc_frame_submit failed (see stderr)")


def frames_wait(timing=None):
    """Block until every submitted frame is complete (rc_frames_wait)."""
    t = RcTiming()
    if hip_lib().rc_frames_wait(ctypes.byref(t)) != 0:
        raise RuntimeError(f"rc_frames_wait failed: {t.frames_failed} of {t.frames_checked} "
                           "frames' carry hand-offs failed (see stderr)")
    if timing is not None:
        timing.update({k: getattr(t, k) for k, _ in RcTiming._fields_})


SPIN_SITES = ("team_handoff", "phase_c_carry_in", "ready_queue", "helper_queue")


def resolver_stats(lone=False):
    """Resolver diagnostics (rc_resolver_stats_get): the last rc_frames_wait window (frames in
    flight), or with lone=True the one-frame-at-a-time renders read back since the last such
    call.  A dict; spin waits by site in microseconds."""
    st = RcResolverStats()
    if hip_lib().rc_resolver_stats_get(1 if lone else 0, ctypes.byref(st)) != 0:
        raise RuntimeError("rc_resolver_stats_get failed")
    d = {k: getattr(st, k) for k, _ in RcResolverStats._fields_ if k not in ("pad", "spin_wait_us_max")}
    d["spin_wait_us_max"] = {n: round(st.spin_wait_us_max[i], 1) for i, n in enumerate(SPIN_SITES)}
    return d


def lone_frames_check():
    """Synchronise the device and read back every one-frame-at-a-time parity frame's hand-off
    words since the previous check (rc_lone_frames_check): {"checked": n, "failed": 0}; raises
    if a frame failed."""
    c, f = ctypes.c_int64(0), ctypes.c_int64(0)
    rc = hip_lib().rc_lone_frames_check(ctypes.byref(c), ctypes.byref(f))
    if rc != 0:
        raise RuntimeError(f"rc_lone_frames_check: {f.value} of {c.value} frames failed (see stderr)")
    return {"checked": c.value, "failed": f.value}


def inject_error(nth_frame):
    """Test aid (rc_debug_inject_error): the nth_frame-th parity frame from now (0 = next)
    fails its carry hand-off as a timed-out spin would; -1 cancels."""
    if hip_lib().rc_debug_inject_error(int(nth_frame)) != 0:
        raise ValueError(nth_frame)


def scatter_selftest(ndep, seed=0, skip=0):
    """Test aid (rc_debug_scatter_selftest, no GPU): rc_render's in-frame scatter against a
    host writer thread; returns the number of wrong pixmap bytes or the failure status."""
    lib = hip_lib()
    lib.rc_debug_scatter_selftest.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.c_int]
    return lib.rc_debug_scatter_selftest(int(ndep), int(seed), int(skip))


def write_p3(img, path):
    """ppm_WriteOutP3 (C/ppm.c:168-184, the product's byte-identical writer) of an [H, W, 3]
    uint8 image into `path`."""
    lib = front_lib()
    h, w, _ = img.shape
    img = np.ascontiguousarray(img)
    p = PPMFormat(w, h, w * h * 3, 255, 0, None, img.ctypes.data)
    f = _libc.fopen(os.fsencode(path), b"wb")
    if not f:
        raise OSError(path)
    try:
        lib.ppm_WriteOutP3(p, ctypes.c_void_p(f))
    finally:
        _libc.fclose(f)


def p3_bytes(img):
    """The P3 file the reference would write for img (C/ppm.c:168-184), produced by the
    product writer into memory (open_memstream)."""
    lib = front_lib()
    h, w, _ = img.shape
    img = np.ascontiguousarray(img)
    p = PPMFormat(w, h, w * h * 3, 255, 0, None, img.ctypes.data)
    buf, size = ctypes.c_void_p(), ctypes.c_size_t()
    f = _libc.open_memstream(ctypes.byref(buf), ctypes.byref(size))
    if not f:
        raise MemoryError("open_memstream")
    lib.ppm_WriteOutP3(p, ctypes.c_void_p(f))
    _libc.fclose(f)
    try:
        return ctypes.string_at(buf, size.value)
    finally:
        _libc.free(buf)


def p3_md5(img):
    """md5 of the P3 file the reference would write for img (C/ppm.c:168-184)."""
    import hashlib
    return hashlib.md5(p3_bytes(img)).hexdigest()


def pipe_reset():
    """Wait for every frame, then release the frame pipeline (rc_pipe_reset); the next
    frame_submit rebuilds it from the current RC_PIPE_* environment."""
    if hip_lib().rc_pipe_reset() != 0:
        raise RuntimeError("rc_pipe_reset failed: a resolver hand-off timed out (see stderr)")


def last_kernel_ms():
    return hip_lib().rc_last_kernel_ms()


def profile_begin():
    """Start a per-phase kernel timing window on the current device (rc_profile_begin)."""
    if hip_lib().rc_profile_begin() != 0:
        raise RuntimeError("rc_profile_begin failed")


def profile_end():
    """Close the window: per-phase kernel times (ms) averaged over the renders inside it."""
    st = RcPhaseStats()
    if hip_lib().rc_profile_end(ctypes.byref(st)) != 0:
        raise RuntimeError("rc_profile_end failed")
    return {k: getattr(st, k) for k, _ in RcPhaseStats._fields_}


def encode_p3(img):
    """The reference P3 byte stream (C/ppm.c:168-184) of an [H, W, 3] uint8 image."""
    h, w, _ = img.shape
    table = [f"{v}\n".encode() for v in range(256)]
    body = b"".join(table[v] for v in img.reshape(-1).tolist())
    return f"P3\n{w} {h} \n255\n".encode() + body


def version():
    return hip_lib().rc_version().decode()


# ------------------------------------------------------------- multi-GPU row shards --
XFER = {"auto": 0, "rccl": 1, "copy": 2}
GROUP_ID_BYTES = 128


class Group:
    """Row-sharded rendering over several GPUs (rc_group / rc_render_sharded):
    row y -> rank y % G, RCCL gathers to rank 0; parity adds the DEP-entry gather, the
    carry resolver on the root and the carry-in scatter.  `Group.local([0, 1, 2])` drives all
    ranks from this process; `Group.rank(world, rank, uid, device)` is one rank of a
    one-process-per-GPU job (uid from `Group.unique_id()` on rank 0, shared by the caller)."""

    def __init__(self, handle):
        if not handle:
            raise RuntimeError("rc_group creation failed (see stderr)")
        self._h = handle

    @staticmethod
    def unique_id():
        buf = ctypes.create_string_buffer(GROUP_ID_BYTES)
        if hip_lib().rc_group_unique_id(buf) != 0:
            raise RuntimeError("rc_group_unique_id failed")
        return buf.raw

    @classmethod
    def local(cls, devices, transport="auto"):
        arr = (ctypes.c_int * len(devices))(*devices)
        return cls(hip_lib().rc_group_create_local(len(devices), arr, XFER[transport]))

    @classmethod
    def rank(cls, world, rank, uid, device):
        assert len(uid) == GROUP_ID_BYTES
        return cls(hip_lib().rc_group_create_rank(world, rank, uid, device))

    @property
    def size(self):
        return hip_lib().rc_group_size(self._h)

    @property
    def transport(self):
        return {1: "rccl", 2: "copy"}[hip_lib().rc_group_transport(self._h)]

    def render(self, scene, width, height, d_image_ptr=None, depth=6, mode="parity",
               timing=None):
        """Collective render; the root's image lands at d_image_ptr (W*H*3 B on rank 0's
        device)."""
        opt = options(depth, mode)
        t = RcTiming()
        rc = hip_lib().rc_render_sharded(self._h, scene.packed(), width, height, ctypes.byref(opt),
                                         ctypes.c_void_p(d_image_ptr or 0), ctypes.byref(t))
        if rc != 0:
            raise RuntimeError("rc_render_sharded failed (see stderr)")
        if timing is not None:
            timing.update({k: getattr(t, k) for k, _ in RcTiming._fields_})

    def stats(self):
        st = RcShardStats()
        if hip_lib().rc_group_last_stats(self._h, ctypes.byref(st)) != 0:
            raise RuntimeError("rc_group_last_stats failed")
        return {k: getattr(st, k) for k, _ in RcShardStats._fields_}

    def rank_stats(self, rank):
        """One rank's own timeline of the last render (rc_group_rank_stats), or None when this
        process does not drive that rank."""
        st = RcRankStats()
        if hip_lib().rc_group_rank_stats(self._h, int(rank), ctypes.byref(st)) != 0:
            return None
        return {k: getattr(st, k) for k, _ in RcRankStats._fields_}

    def debug_bound(self, per_rank):
        """Test aid (rc_group_debug_bound): the fixed-size entry exchange's per-rank bound."""
        if hip_lib().rc_group_debug_bound(self._h, int(per_rank)) != 0:
            raise ValueError(per_rank)

    def close(self):
        if self._h:
            hip_lib().rc_group_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def row_shard(height, rank, world):
    """Rows of rank `rank` under the row-cyclic partition (row y -> rank y % world):
    (row0, row_step, nrows).  Contiguous blocks are 1.7-2.1x imbalanced on the reference
    scenes at 8 ranks; cyclic rows are within ~2%."""
    return rank, world, (height - rank + world - 1) // world


def deinterleave(gathered, height):
    """Undo the row-cyclic partition: image row y = gathered[y % world][y // world] (the
    host-side statement of k_deinterleave, for the CPU protocol tests)."""
    world, rows_max, w, c = gathered.shape
    full = gathered.permute(1, 0, 2, 3).reshape(rows_max * world, w, c)
    return full[:height]
