"""ctypes mirror of include/bdpt/bdpt.h plus thin Python helpers (plumbing for tests / bench).

The product is libbdpt_amd.so (HIP kernels + C-ABI) and the C++ `pathtracer` CLI next to it;
this module only marshals scene descriptions and frames across the C-ABI. It never falls back
to a CPU path: if the shared library is missing, `load_library()` raises.

Reference interfaces mirrored (see include/bdpt/bdpt.h for the full map):
  BidirectionalPathTracer::raytrace_pixel  src/pathtracer/bidirection.cpp:503-542
  RaytracedRenderer::raytrace_tile         src/pathtracer/raytraced_renderer.cpp:595-620
"""
from __future__ import annotations

import ctypes as C
import json
import os
from typing import Optional, Sequence

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libbdpt_amd.so")

BDPT_OK = 0
BDPT_E_INVALID = -1
BDPT_E_UNSUPPORTED = -2
BDPT_E_DEVICE = -3
BDPT_E_NOMEM = -4

PRIM_TRIANGLE, PRIM_SPHERE = 0, 1
MAT_DIFFUSE, MAT_EMISSION, MAT_MIRROR, MAT_GLASS, MAT_REFRACTION, MAT_MICROFACET = range(6)
LIGHT_AREA, LIGHT_POINT, LIGHT_OTHER, LIGHT_HEMISPHERE, LIGHT_DIRECTIONAL = 0, 1, 2, 3, 4
FRAME_SAMPLE, FRAME_EYE, FRAME_LIGHT = 0, 1, 2

_MAT_NAMES = {"diffuse": MAT_DIFFUSE, "emission": MAT_EMISSION, "mirror": MAT_MIRROR,
              "glass": MAT_GLASS, "refraction": MAT_REFRACTION, "microfacet": MAT_MICROFACET}


class Material(C.Structure):
    _fields_ = [("type", C.c_int32), ("a", C.c_double * 3), ("b", C.c_double * 3),
                ("ior", C.c_double), ("roughness", C.c_double)]


class Light(C.Structure):
    _fields_ = [("type", C.c_int32), ("radiance", C.c_double * 3), ("position", C.c_double * 3),
                ("direction", C.c_double * 3), ("dim_x", C.c_double * 3),
                ("dim_y", C.c_double * 3), ("area", C.c_double)]


class Camera(C.Structure):
    _fields_ = [("pos", C.c_double * 3), ("c2w", C.c_double * 9), ("w2c", C.c_double * 9),
                ("hfov_deg", C.c_double), ("vfov_deg", C.c_double), ("nclip", C.c_double),
                ("fclip", C.c_double)]


class EnvMapDesc(C.Structure):
    """bdpt_envmap: the -e environment map (HDRImageBuffer data[w*j + i], row 0 = theta 0)."""
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("rgb", C.POINTER(C.c_float))]


class SceneDesc(C.Structure):
    _fields_ = [("nprim", C.c_int32), ("prim_type", C.POINTER(C.c_int32)),
                ("prim_geom", C.POINTER(C.c_double)), ("prim_mat", C.POINTER(C.c_int32)),
                ("nmat", C.c_int32), ("mats", C.POINTER(Material)),
                ("nlight", C.c_int32), ("lights", C.POINTER(Light)), ("camera", Camera),
                ("envmap", C.POINTER(EnvMapDesc))]


class Params(C.Structure):
    _fields_ = [("width", C.c_int32), ("height", C.c_int32), ("spp", C.c_int32),
                ("max_depth", C.c_int32), ("seed", C.c_uint64), ("samples_per_lane", C.c_int32),
                ("device", C.c_int32), ("collect_stats", C.c_int32), ("pipeline", C.c_int32),
                ("russian_roulette", C.c_int32), ("integrator", C.c_int32),
                ("ns_area_light", C.c_int32), ("samples_per_batch", C.c_int32),
                ("max_tolerance", C.c_float), ("direct_hemisphere_sample", C.c_int32),
                ("lens_radius", C.c_double), ("focal_distance", C.c_double),
                ("reserved", C.c_int32 * 4)]


INTEGRATOR_BDPT, INTEGRATOR_PT = 0, 1


class Tile(C.Structure):
    _fields_ = [("x0", C.c_int32), ("y0", C.c_int32), ("w", C.c_int32), ("h", C.c_int32)]


PIPELINE_AUTO, PIPELINE_MEGAKERNEL = 0, 1
PIPELINE_WAVEFRONT = 2   # retired in round 5: bdpt_create rejects it


class Stats(C.Structure):
    _fields_ = [("samples", C.c_uint64), ("rays", C.c_uint64), ("closest_rays", C.c_uint64),
                ("shadow_rays", C.c_uint64), ("node_visits", C.c_uint64),
                ("tri_tests", C.c_uint64), ("sph_tests", C.c_uint64), ("hits", C.c_uint64),
                ("last_kernel_ms", C.c_double), ("bvh_nodes", C.c_uint64),
                ("bvh_depth", C.c_uint64), ("lds_node_visits", C.c_uint64),
                ("lds_mode", C.c_int32), ("reserved0", C.c_int32),
                ("env_samples", C.c_uint64), ("env_lookups", C.c_uint64), ("env_pdf_lookups", C.c_uint64)]


class Scene:
    """Owns numpy arrays backing a SceneDesc (keeps them alive while the desc is used)."""

    def __init__(self, prim_type, prim_geom, prim_mat, mats, lights, camera: dict,
                 width: int = 0, height: int = 0, envmap: Optional[np.ndarray] = None):
        self.prim_type = np.ascontiguousarray(prim_type, dtype=np.int32)
        self.prim_geom = np.ascontiguousarray(prim_geom, dtype=np.float64).reshape(-1, 18)
        self.prim_mat = np.ascontiguousarray(prim_mat, dtype=np.int32)
        self.mats = (Material * max(1, len(mats)))()
        for i, m in enumerate(mats):
            self.mats[i] = m
        self.nmat = len(mats)
        self.lights = (Light * max(1, len(lights)))()
        for i, l in enumerate(lights):
            self.lights[i] = l
        self.nlight = len(lights)
        self.camera = camera
        self.width, self.height = width, height
        self.set_envmap(envmap)

    def set_envmap(self, envmap: Optional[np.ndarray]) -> None:
        """Environment map (H, W, 3) float32, row 0 = theta 0 (+y); None removes it."""
        if envmap is None:
            self.envmap = None
            self._env_desc = None
            return
        self.envmap = np.ascontiguousarray(envmap, dtype=np.float32).reshape(
            envmap.shape[0], envmap.shape[1], 3)
        e = EnvMapDesc()
        e.height, e.width = self.envmap.shape[0], self.envmap.shape[1]
        e.rgb = self.envmap.ctypes.data_as(C.POINTER(C.c_float))
        self._env_desc = e

    def load_camera(self, path: str, focal_distance: float = 4.7, lens_radius: float = 0.0):
        """Application::load_camera -> Camera::load_settings (application.h:114-116, camera.cpp:172-186):
        the -c camera-settings file through bdpt_camera_load_settings_lens (w2c kept, as the reference
        does not recompute it). Returns the thin-lens settings the camera then holds: the file's
        focalDistance and lensRadius, which replace the ones passed in (the config's -d / -b,
        set_camera, raytraced_renderer.cpp:141-142) — give them to PathTracer(...)."""
        lib = load_library()
        cam = self.desc().camera
        fd, lr = C.c_double(focal_distance), C.c_double(lens_radius)
        _check(lib.bdpt_camera_load_settings_lens(os.fsencode(path), C.byref(cam), C.byref(fd), C.byref(lr)), lib)
        c = dict(self.camera)
        c["pos"] = list(cam.pos)
        c["c2w_cols"] = [list(cam.c2w[3 * k:3 * k + 3]) for k in range(3)]
        c["hFov"], c["vFov"], c["nClip"], c["fClip"] = cam.hfov_deg, cam.vfov_deg, cam.nclip, cam.fclip
        self.camera = c
        return fd.value, lr.value

    @property
    def nprim(self) -> int:
        return int(self.prim_type.shape[0])

    def desc(self) -> SceneDesc:
        d = SceneDesc()
        d.nprim = self.nprim
        d.prim_type = self.prim_type.ctypes.data_as(C.POINTER(C.c_int32))
        d.prim_geom = self.prim_geom.ctypes.data_as(C.POINTER(C.c_double))
        d.prim_mat = self.prim_mat.ctypes.data_as(C.POINTER(C.c_int32))
        d.nmat = self.nmat
        d.mats = C.cast(self.mats, C.POINTER(Material))
        d.nlight = self.nlight
        d.lights = C.cast(self.lights, C.POINTER(Light))
        cam = Camera()
        c = self.camera
        cam.pos[:] = c["pos"]
        cam.c2w[:] = [v for col in c["c2w_cols"] for v in col]
        cam.w2c[:] = [v for col in c["w2c_cols"] for v in col]
        cam.hfov_deg, cam.vfov_deg = c["hFov"], c["vFov"]
        cam.nclip, cam.fclip = c["nClip"], c["fClip"]
        d.camera = cam
        d.envmap = C.pointer(self._env_desc) if self._env_desc is not None else None
        return d


def scene_from_json(js) -> Scene:
    """Scene from the JSON dump format (tests/golden/scenes/*.json, written by
    oracle/_ref/ref_driver or by the C++ loader's --dump-scene)."""
    if isinstance(js, (str, os.PathLike)):
        with open(js) as f:
            js = json.load(f)
    tris, sphs = js["triangles"], js["spheres"]
    order = js.get("prim_order")  # list of ["t", i] / ["s", i] in scene order, if present
    if order is None:
        order = [("t", i) for i in range(len(tris))] + [("s", i) for i in range(len(sphs))]
    ptype, geom, pmat = [], [], []
    for kind, i in order:
        g = [0.0] * 18
        if kind == "t":
            t = tris[i]
            g[:18] = [x for v in t[:6] for x in v]
            ptype.append(PRIM_TRIANGLE)
            pmat.append(t[6])
        else:
            s = sphs[i]
            g[0:3] = s[0]
            g[3] = s[1]
            ptype.append(PRIM_SPHERE)
            pmat.append(s[2])
        geom.append(g)
    mats = []
    for m in js["materials"]:
        M = Material()
        M.type = _MAT_NAMES.get(m["type"], -1)
        if m["type"] in ("diffuse", "mirror"):
            M.a[:] = m["reflectance"]
        elif m["type"] == "emission":
            M.a[:] = m["radiance"]
        elif m["type"] == "glass":
            M.a[:] = m["reflectance"]
            M.b[:] = m["transmittance"]
            M.ior, M.roughness = m["ior"], m.get("roughness", 0.0)
        elif m["type"] == "refraction":
            M.b[:] = m["transmittance"]
            M.ior, M.roughness = m["ior"], m.get("roughness", 0.0)
        elif m["type"] == "microfacet" and "eta" in m:
            M.a[:], M.b[:], M.roughness = m["eta"], m["k"], m["alpha"]
        mats.append(M)
    lights = []
    for l in js["lights"]:
        L = Light()
        if l["type"] == "area":
            L.type = LIGHT_AREA
            L.radiance[:], L.position[:] = l["radiance"], l["position"]
            L.direction[:], L.dim_x[:], L.dim_y[:] = l["direction"], l["dim_x"], l["dim_y"]
            L.area = l["area"]
        elif l["type"] == "point":
            L.type = LIGHT_POINT
            L.radiance[:], L.position[:] = l["radiance"], l["position"]
        elif l["type"] == "hemisphere":          # an ambient light (InfiniteHemisphereLight)
            L.type = LIGHT_HEMISPHERE
            L.radiance[:] = l["radiance"]
        elif l["type"] == "directional":         # DirectionalLight: direction = dirToLight
            L.type = LIGHT_DIRECTIONAL
            L.radiance[:], L.direction[:] = l["radiance"], l["direction"]
        else:
            L.type = LIGHT_OTHER
        lights.append(L)
    cam = js["camera"]
    return Scene(ptype, geom, pmat, mats, lights, cam, cam.get("screenW", 0), cam.get("screenH", 0))


def load_dae(path: str, width: int = 0, height: int = 0, dump_json: str = None) -> Scene:
    """Scene from a COLLADA file through the library's host loader (bdpt_dae_load: ColladaParser
    + Application::load semantics). width/height > 0 apply the -r W H camera retarget."""
    lib = load_library()
    h = C.c_void_p()
    _check(lib.bdpt_dae_load(os.fsencode(path), width, height, C.byref(h)), lib)
    try:
        if dump_json:
            _check(lib.bdpt_dae_dump_json(h, os.fsencode(dump_json)), lib)
        d = SceneDesc()
        _check(lib.bdpt_dae_get_desc(h, C.byref(d)), lib)
        n = d.nprim
        ptype = np.ctypeslib.as_array(d.prim_type, shape=(n,)).copy() if n else np.zeros(0, np.int32)
        geom = np.ctypeslib.as_array(d.prim_geom, shape=(n * 18,)).copy() if n else np.zeros(0)
        pmat = np.ctypeslib.as_array(d.prim_mat, shape=(n,)).copy() if n else np.zeros(0, np.int32)
        mats = [Material.from_buffer_copy(d.mats[i]) for i in range(d.nmat)]
        lights = [Light.from_buffer_copy(d.lights[i]) for i in range(d.nlight)]
        c = d.camera
        cam = {"pos": list(c.pos), "c2w_cols": [list(c.c2w[3 * k:3 * k + 3]) for k in range(3)],
               "w2c_cols": [list(c.w2c[3 * k:3 * k + 3]) for k in range(3)],
               "hFov": c.hfov_deg, "vFov": c.vfov_deg, "nClip": c.nclip, "fClip": c.fclip}
        return Scene(ptype, geom, pmat, mats, lights, cam, width, height)
    finally:
        lib.bdpt_dae_free(h)


def retarget_camera(scene: Scene, width: int, height: int) -> Scene:
    """Camera::set_screen_size (camera.cpp:83-89): screenDist fixed, FOV follows the frame size
    (the reference's FOV quirk)."""
    import math
    c = dict(scene.camera)
    sd = c["screenDist"]
    c["hFov"] = 2 * math.degrees(math.atan(float(width) / (2 * sd)))
    c["vFov"] = 2 * math.degrees(math.atan(float(height) / (2 * sd)))
    c["screenW"], c["screenH"] = width, height
    out = Scene(scene.prim_type, scene.prim_geom, scene.prim_mat,
                [scene.mats[i] for i in range(scene.nmat)],
                [scene.lights[i] for i in range(scene.nlight)], c, width, height, scene.envmap)
    return out


def load_exr(path: str) -> np.ndarray:
    """OpenEXR environment map through the library's reader (bdpt_exr_load: load_exr,
    main.cpp:40-77): (H, W, 3) float32, row 0 = top."""
    lib = load_library()
    w, h = C.c_int32(), C.c_int32()
    ptr = C.POINTER(C.c_float)()
    _check(lib.bdpt_exr_load(os.fsencode(path), C.byref(w), C.byref(h), C.byref(ptr)), lib)
    try:
        return np.ctypeslib.as_array(ptr, shape=(h.value, w.value, 3)).copy()
    finally:
        lib.bdpt_exr_free(ptr)


# ------------------------------------------------------------------------------------------------
_lib = None


def load_library(path: Optional[str] = None) -> C.CDLL:
    """Loads libbdpt_amd.so (the HIP product). Raises if it is missing — there is no fallback."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError(f"libbdpt_amd.so not built ({p}); run __graft_entry__.build()")
    lib = C.CDLL(p)
    lib.bdpt_abi_version.restype = C.c_int
    lib.bdpt_last_error.restype = C.c_char_p
    lib.bdpt_create.argtypes = [C.POINTER(SceneDesc), C.POINTER(Params), C.POINTER(C.c_void_p)]
    lib.bdpt_destroy.argtypes = [C.c_void_p]
    lib.bdpt_destroy.restype = None
    lib.bdpt_set_stream.argtypes = [C.c_void_p, C.c_void_p]
    lib.bdpt_clear.argtypes = [C.c_void_p]
    lib.bdpt_render.argtypes = [C.c_void_p, C.POINTER(Tile), C.c_int32, C.c_int32, C.c_int32]
    lib.bdpt_sync.argtypes = [C.c_void_p]
    lib.bdpt_read_frame.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_float)]
    lib.bdpt_frame_device_ptr.argtypes = [C.c_void_p, C.c_int32, C.POINTER(C.c_void_p)]
    lib.bdpt_copy_frame.argtypes = [C.c_void_p, C.c_int32, C.c_void_p]
    lib.bdpt_get_stats.argtypes = [C.c_void_p, C.POINTER(Stats)]
    lib.bdpt_read_sample_counts.argtypes = [C.c_void_p, C.POINTER(C.c_int32)]
    lib.bdpt_trace_rays.argtypes = [C.c_void_p, C.POINTER(C.c_float), C.c_int32, C.c_int32,
                                    C.POINTER(C.c_float), C.POINTER(C.c_int32)]
    lib.bdpt_dae_load.argtypes = [C.c_char_p, C.c_int32, C.c_int32, C.POINTER(C.c_void_p)]
    lib.bdpt_dae_get_desc.argtypes = [C.c_void_p, C.POINTER(SceneDesc)]
    lib.bdpt_dae_dump_json.argtypes = [C.c_void_p, C.c_char_p]
    lib.bdpt_dae_free.argtypes = [C.c_void_p]
    lib.bdpt_read_frame_rect.argtypes = [C.c_void_p, C.c_int32, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                         C.POINTER(C.c_float)]
    lib.bdpt_camera_load_settings.argtypes = [C.c_char_p, C.POINTER(Camera)]
    lib.bdpt_camera_load_settings_lens.argtypes = [C.c_char_p, C.POINTER(Camera), C.POINTER(C.c_double),
                                                   C.POINTER(C.c_double)]
    lib.bdpt_dae_free.restype = None
    lib.bdpt_exr_load.argtypes = [C.c_char_p, C.POINTER(C.c_int32), C.POINTER(C.c_int32),
                                  C.POINTER(C.POINTER(C.c_float))]
    lib.bdpt_exr_free.argtypes = [C.POINTER(C.c_float)]
    lib.bdpt_exr_free.restype = None
    lib.bdpt_reduce_create.argtypes = [C.POINTER(C.c_void_p), C.c_int32, C.POINTER(C.c_void_p)]
    lib.bdpt_reduce_frames.argtypes = [C.c_void_p, C.c_int32]
    lib.bdpt_reduce_ranks.argtypes = [C.c_void_p]
    lib.bdpt_reduce_destroy.argtypes = [C.c_void_p]
    lib.bdpt_reduce_destroy.restype = None
    if path is None:
        _lib = lib
    return lib


class BDPTError(RuntimeError):
    pass


def _check(rc: int, lib) -> None:
    if rc != BDPT_OK:
        msg = lib.bdpt_last_error()
        raise BDPTError(f"bdpt error {rc}: {msg.decode() if msg else ''}")


class BidirectionalPathTracer:
    """Host-side mirror of the reference's PathTracer entry points over the C-ABI
    (pathtracer.h:36-69; bidirection.h:51-92). One instance = one device context."""

    def __init__(self, scene: Scene, width: int, height: int, spp: int, max_depth: int,
                 seed: int = 5489, device: int = 0, samples_per_lane: int = 0,
                 collect_stats: bool = False, pipeline: int = PIPELINE_AUTO,
                 russian_roulette: bool = False, _pt: Optional[dict] = None):
        self.lib = load_library()
        self.scene = scene
        self.width, self.height, self.spp, self.max_depth = width, height, spp, max_depth
        p = Params()
        p.width, p.height, p.spp, p.max_depth = width, height, spp, max_depth
        p.seed, p.samples_per_lane, p.device = seed, samples_per_lane, device
        p.collect_stats = 1 if collect_stats else 0
        p.pipeline = pipeline
        p.russian_roulette = 1 if russian_roulette else 0
        if _pt is not None:
            p.integrator = INTEGRATOR_PT
            p.ns_area_light = _pt["ns_area_light"]
            p.samples_per_batch = _pt["samples_per_batch"]
            p.max_tolerance = _pt["max_tolerance"]
            p.direct_hemisphere_sample = 1 if _pt["direct_hemisphere_sample"] else 0
            p.lens_radius, p.focal_distance = _pt["lens_radius"], _pt["focal_distance"]
        self._desc = scene.desc()
        self._reducers = []   # FrameReducers over this context: closed before it is destroyed
        ctx = C.c_void_p()
        _check(self.lib.bdpt_create(C.byref(self._desc), C.byref(p), C.byref(ctx)), self.lib)
        self.ctx = ctx

    def close(self) -> None:
        for red in list(getattr(self, "_reducers", ())):
            red.close()
        if getattr(self, "ctx", None):
            self.lib.bdpt_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_stream(self, stream_handle: int) -> None:
        _check(self.lib.bdpt_set_stream(self.ctx, C.c_void_p(stream_handle)), self.lib)

    def clear(self) -> None:
        _check(self.lib.bdpt_clear(self.ctx), self.lib)

    def raytrace_tiles(self, tiles: Sequence[tuple] = (), spp_begin: int = 0,
                       spp_count: Optional[int] = None) -> None:
        n = len(tiles)
        arr = (Tile * max(1, n))()
        for i, t in enumerate(tiles):
            arr[i] = Tile(*t)
        cnt = self.spp - spp_begin if spp_count is None else spp_count
        _check(self.lib.bdpt_render(self.ctx, arr if n else None, n, spp_begin, cnt), self.lib)

    def raytrace_tile(self, x0: int, y0: int, w: int, h: int) -> None:
        self.raytrace_tiles([(x0, y0, w, h)])

    def raytrace_pixel(self, x: int, y: int) -> None:
        self.raytrace_tiles([(x, y, 1, 1)])

    def sync(self) -> None:
        _check(self.lib.bdpt_sync(self.ctx), self.lib)

    def read_frame(self, which: int = FRAME_SAMPLE) -> np.ndarray:
        out = np.empty((self.height, self.width, 3), dtype=np.float32)
        _check(self.lib.bdpt_read_frame(self.ctx, which, out.ctypes.data_as(C.POINTER(C.c_float))),
               self.lib)
        return out

    def frame_device_ptr(self, which: int = FRAME_SAMPLE) -> int:
        p = C.c_void_p()
        _check(self.lib.bdpt_frame_device_ptr(self.ctx, which, C.byref(p)), self.lib)
        return int(p.value or 0)

    def copy_frame(self, which: int, dst_device_ptr: int) -> None:
        _check(self.lib.bdpt_copy_frame(self.ctx, which, C.c_void_p(dst_device_ptr)), self.lib)

    def read_sample_counts(self) -> np.ndarray:
        """sampleCountBuffer (pathtracer.h:94): (H, W) int32, row 0 = bottom."""
        out = np.empty((self.height, self.width), dtype=np.int32)
        _check(self.lib.bdpt_read_sample_counts(self.ctx, out.ctypes.data_as(C.POINTER(C.c_int32))),
               self.lib)
        return out

    def stats(self) -> Stats:
        s = Stats()
        _check(self.lib.bdpt_get_stats(self.ctx, C.byref(s)), self.lib)
        return s

    def trace_rays(self, rays: np.ndarray, any_hit: bool = False):
        rays = np.ascontiguousarray(rays, dtype=np.float32).reshape(-1, 8)
        n = rays.shape[0]
        t = np.empty(n, dtype=np.float32)
        prim = np.empty(n, dtype=np.int32)
        _check(self.lib.bdpt_trace_rays(self.ctx, rays.ctypes.data_as(C.POINTER(C.c_float)), n,
                                        1 if any_hit else 0, t.ctypes.data_as(C.POINTER(C.c_float)),
                                        prim.ctypes.data_as(C.POINTER(C.c_int32))), self.lib)
        return t, prim


class PathTracer(BidirectionalPathTracer):
    """The reference's unidirectional integrator (PathTracer, pathtracer.cpp:47-340) on the GPU:
    next-event estimation (-l samples per area light, or -H hemisphere sampling), adaptive
    sampling in batches (-a batch tol), thin lens (-b, -d), roulette at max_depth 0, the
    environment light, MicrofacetBSDF. Defaults are AppConfig's (application.h:45-65).
    raytrace_tiles() renders whole pixels (spp_begin 0, all ns_aa samples)."""

    def __init__(self, scene: Scene, width: int, height: int, spp: int, max_depth: int,
                 seed: int = 5489, device: int = 0, ns_area_light: int = 1,
                 samples_per_batch: int = 32, max_tolerance: float = 0.05,
                 direct_hemisphere_sample: bool = False, lens_radius: float = 0.0,
                 focal_distance: float = 4.7, collect_stats: bool = False):
        super().__init__(scene, width, height, spp, max_depth, seed=seed, device=device,
                         collect_stats=collect_stats,
                         _pt=dict(ns_area_light=ns_area_light, samples_per_batch=samples_per_batch,
                                  max_tolerance=max_tolerance,
                                  direct_hemisphere_sample=direct_hemisphere_sample,
                                  lens_radius=lens_radius, focal_distance=focal_distance))


class FrameReducer:
    """The C-ABI's multi-GPU frame reduce (bdpt_reduce_*, ABI v9) over renderers in ONE process —
    the CLI's -g N: one RCCL communicator clique over their distinct devices (contexts sharing a
    device are summed on it first), and per reduce(root) one grouped ncclReduce of every
    renderer's eye and light frames into the root renderer's. Afterwards root.read_frame() is the
    whole image; the others' frames are unchanged. Closing any of its renderers closes the reducer
    first (bdpt_reduce_destroy then touches no context)."""

    def __init__(self, renderers: Sequence["BidirectionalPathTracer"]):
        self.lib = load_library()
        self.renderers = list(renderers)
        if any(not getattr(r, "ctx", None) for r in self.renderers):
            raise BDPTError("FrameReducer: a renderer is closed")
        arr = (C.c_void_p * len(self.renderers))(*[r.ctx.value for r in self.renderers])
        h = C.c_void_p()
        _check(self.lib.bdpt_reduce_create(arr, len(self.renderers), C.byref(h)), self.lib)
        self.h = h
        for r in self.renderers:   # a renderer's close() closes its reducers first
            r._reducers.append(self)

    @property
    def ranks(self) -> int:
        """RCCL ranks of the communicator (distinct devices)"""
        return int(self.lib.bdpt_reduce_ranks(self.h))

    def reduce(self, root: int = 0) -> None:
        if not getattr(self, "h", None):
            raise BDPTError("FrameReducer is closed")
        _check(self.lib.bdpt_reduce_frames(self.h, root), self.lib)

    def close(self) -> None:
        if getattr(self, "h", None):
            self.lib.bdpt_reduce_destroy(self.h)
            self.h = None
        for r in getattr(self, "renderers", ()):
            if self in getattr(r, "_reducers", ()):
                r._reducers.remove(self)

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# --- multi-GPU: one process per GPU under torch.distributed ---------
# Pixel-samples are independent except the t = 1 light-tracing splats, which land anywhere
# (bidirection.cpp:457-466), so a frame cannot be split into tiles and gathered: the ranks split
# the SAMPLE range of every pixel and the W*H*3 frames are summed. The RNG is keyed by the global
# sample index, so the sum equals one render of all the samples up to fp32 summation order.


def rank_sample_range(step: int, rank: int, world: int, spp: int, scaling: str = "strong"):
    """Global sample indices [begin, begin + count) that `rank` renders in `step`.
    strong: the step's fixed render of `spp` samples per pixel is split across the ranks;
    weak: every rank renders a fresh `spp` of its own. Either way every (step, rank) owns a
    disjoint range, so the summed frames equal one render of all those samples."""
    if scaling == "strong":
        lo, hi = spp * rank // world, spp * (rank + 1) // world
        return step * spp + lo, hi - lo
    return (step * world + rank) * spp, spp


class ShardedRender:
    """One rank's part of a multi-GPU render: per step, render this rank's sample range of the
    whole frame (bdpt_render, async on the context's stream), copy the sample frame into `frame`
    (a float32 tensor of W*H*3 on this rank's device, bdpt_copy_frame) and sum `frame` over the
    ranks with ONE all-reduce — the only collective (RCCL over xGMI with the "nccl" backend; gloo
    takes device tensors for all_reduce too, which is how two ranks can share one GPU in tests).
    A renderer needs raytrace_tiles(tiles, spp_begin, spp_count) and copy_frame(which, ptr) —
    BidirectionalPathTracer, or any object with the same two calls.
    With a device `frame`, the renderer's context is put on torch's current stream of that device
    (set_stream), so the render, the frame copy and the collective (which torch orders after that
    stream's work) run in order without a host sync; on the null stream reduce() syncs the
    context before the collective instead."""

    def __init__(self, pt, frame, rank: int, world: int, spp: int, scaling: str = "strong", dist=None,
                 group=None):
        self.pt, self.frame = pt, frame
        self._host_sync = False
        if getattr(frame, "is_cuda", False) and hasattr(pt, "set_stream"):
            import torch
            handle = torch.cuda.current_stream(frame.device).cuda_stream
            if handle:
                pt.set_stream(handle)
            else:   # the null stream: handle 0 would select the context's own stream
                self._host_sync = True
        self.rank, self.world, self.spp, self.scaling = rank, world, spp, scaling
        self.dist, self.group = dist, group

    def samples(self, step: int) -> int:
        """sample indices per pixel this rank renders in `step`"""
        return rank_sample_range(step, self.rank, self.world, self.spp, self.scaling)[1]

    def render(self, step: int) -> None:
        base, n = rank_sample_range(step, self.rank, self.world, self.spp, self.scaling)
        if n > 0:
            self.pt.raytrace_tiles([], base, n)

    def reduce(self) -> None:
        self.pt.copy_frame(FRAME_SAMPLE, self.frame.data_ptr())
        if self._host_sync:
            self.pt.sync()
        if self.dist is not None:   # at world size 1 too: the same RCCL call on one rank
            self.dist.all_reduce(self.frame, op=self.dist.ReduceOp.SUM, group=self.group)

    def step(self, step: int) -> None:
        self.render(step)
        self.reduce()

    def gather_floats(self, values, device=None):
        """every rank's `values` (a list of floats), as a list per rank — through all_reduce of a
        zero-padded (world x n) tensor, which both backends take for device tensors"""
        import torch
        v = torch.zeros(self.world, len(values), dtype=torch.float64,
                        device=device if device is not None else self.frame.device)
        v[self.rank] = torch.tensor(values, dtype=torch.float64)
        if self.dist is not None:
            self.dist.all_reduce(v, op=self.dist.ReduceOp.SUM, group=self.group)
        return [[float(x) for x in row] for row in v.cpu()]
