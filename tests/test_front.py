"""CPU tests of the host front end and the C-ABI boundary.

- parse_json (own implementation, libraycast_front.so) builds the same lists as the
  reference's parse_json (C/parse.c, compiled into oracle/_ref/libref_front.so) on every
  fixture scene and on reformatted / edge-case variants;
- malformed scenes give the same stderr message and exit status as the reference binary;
- ppm_WriteOutP3 writes the same bytes as the reference writer (C/ppm.c:168-184);
- both shared libraries export every function include/raycast_hip.h declares;
- the drop-in CLI's argument handling matches C/raycast.c:19-39.
No GPU is touched: everything here exits before the first HIP call."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

from helpers import REF_DIR, ROOT, SCENES, have_ref, rc, scene_path, write_p3

CLI = os.path.join(ROOT, "raytracing-programs_amd", "bin", "raytrace")
REF_FRONT = os.path.join(REF_DIR, "libref_front.so")
FIXTURES = ["simple", "reflection", "quadric", "example2", "example3", "quadric2"]

_libc = ctypes.CDLL(None)
_libc.fopen.restype = ctypes.c_void_p
_libc.fopen.argtypes = [ctypes.c_char_p, ctypes.c_char_p]
_libc.fclose.argtypes = [ctypes.c_void_p]


def _parse_with(lib, path):
    lib.parse_json.argtypes = [ctypes.c_void_p, ctypes.POINTER(rc.JsonDataT)]
    f = _libc.fopen(os.fsencode(path), b"r")
    js = rc.JsonDataT()
    lib.parse_json(f, ctypes.byref(js))
    _libc.fclose(f)
    return js


def _records(js):
    """Node bytes without the `next` pointers: shapes (first 96 B), lights (first 64 B).
    Point lights leave theta/cos_theta/a0/direction unset in the reference (malloc): those
    bytes [36, 60) are compared only for spot lights."""
    out = []
    p = js.shapes_list
    # defined bytes per type: common fields [0, 48), the type's union members, `type` [88, 92)
    union_end = {0: 52, 1: 60, 2: 88}   # sphere radius, plane normal, quadric a..j
    while p:
        b = ctypes.string_at(ctypes.addressof(p.contents), 96)
        t = p.contents.type
        rec = bytearray(b[:union_end.get(t, 48)]) + bytearray(b[88:92])
        if t == 2:
            rec[24:36] = bytes(12)   # add_new_quadric never sets position (C/objects.c:97-127)
        out.append(bytes(rec))
        p = ctypes.cast(p.contents.next, ctypes.POINTER(rc.ShapeT))
    lights = []
    p = js.lights_list
    while p:
        b = bytearray(ctypes.string_at(ctypes.addressof(p.contents), 64))
        if p.contents.type == 0:   # POINT
            b[36:60] = bytes(24)
        lights.append(bytes(b))
        p = ctypes.cast(p.contents.next, ctypes.POINTER(rc.LightT))
    return (js.camera_width, js.camera_height, js.num_shapes, js.num_lights, out, lights)


VARIANTS = {
    # spacing / ordering / defaults the grammar allows (C/parse.c:368-430)
    "tight": "camera,width: 3.0,height: 3.0\n"
             "sphere,radius:2.0,diffuse_color:[1,1,1],specular_color:[1,1,1],position:[0,1,-10],"
             " reflectivity: 0.35, refractivity: 0.3, ior: 2\n"
             "plane,normal:[0,4,0],diffuse_color:[0,1,0], position:[0,-1,0], reflectivity: 0\n"
             "light, color:[2,2,2], theta:0, radial-a2:0.075, radial-a1:0.125, radial-a0:0.125, "
             "position:[1,3,-3]",
    "defaults": "camera, width: 2, height: 2\n"
                "quadric, a: 1, b: 0, c: 1, d: 0, e: 0, f: 0, g: 4, h: 0, i: 10, j: 28, "
                "reflectivity: 0.3\n"
                "sphere, position: [4, 0, -7], radius: 1, reflectivity: 0.3, refractivity: 0, ior: 2\n"
                "light, color: [2, 2, 2], radial-a2: 0.075, radial-a1: 0.125, radial-a0: 0.125, "
                "position: [0, 0, -1], theta: 5, angular-a0: 2, direction: [0, 0, -1]\n",
    "blank_lines": "\ncamera, width: 2, height: 2\n\nsphere, radius: 1.0, diffuse_color: [1, 0, 0], "
                   "position: [0, 0, -5], reflectivity: 0.5, refractivity: 0, ior: 1\n\n"
                   "light, color: [1, 1, 1], radial-a2: 0, radial-a1: 0, radial-a0: 1, "
                   "position: [0, 5, 0]\n\n",
    "multiline_vector": "camera, width: 2, height: 2\nsphere, radius: 1.0, diffuse_color: [1,\n0, 0], "
                        "position: [0, 0, -5], reflectivity: 0.5, refractivity: 0, ior: 1\n",
    # a repeated key counts twice and can stand in for a missing one, which then keeps the
    # previous record's value (C/parse.c:15-37 keeps the scratch values across records)
    "repeated_key": "camera, width: 2, height: 2\n"
                    "sphere, radius: 1.0, position: [0, 0, -5], reflectivity: 0.5, "
                    "refractivity: 0.25, ior: 1\n"
                    "sphere, radius: 1.0, radius: 2.0, position: [0, 1, -5], reflectivity: 0.5, "
                    "ior: 3\n",
}

ERRORS = {
    "no_camera": "sphere, radius: 1.0, position: [0, 0, -5], reflectivity: 0.5, refractivity: 0, ior: 1\n",
    "two_cameras": "camera, width: 2, height: 2\ncamera, width: 2, height: 2\n",
    "camera_field": "camera, width: 2\n",
    "sphere_field": "camera, width: 2, height: 2\nsphere, radius: 1.0, position: [0, 0, -5]\n",
    "sphere_refl": "camera, width: 2, height: 2\nsphere, radius: 1.0, position: [0, 0, -5], "
                   "reflectivity: 1.5, refractivity: 0, ior: 1\n",
    "sphere_refr": "camera, width: 2, height: 2\nsphere, radius: 1.0, position: [0, 0, -5], "
                   "reflectivity: 0.5, refractivity: -1, ior: 1\n",
    "plane_field": "camera, width: 2, height: 2\nplane, normal: [0, 1, 0], reflectivity: 0\n",
    "plane_refl": "camera, width: 2, height: 2\nplane, normal: [0, 1, 0], position: [0, -1, 0], "
                  "reflectivity: 2\n",
    "quadric_field": "camera, width: 2, height: 2\nquadric, a: 1, b: 1, reflectivity: 0\n",
    "quadric_refl": "camera, width: 2, height: 2\nquadric, a: 1, b: 0, c: 1, d: 0, e: 0, f: 0, g: 4, "
                    "h: 0, i: 10, j: 28, reflectivity: -0.5\n",
    "light_field": "camera, width: 2, height: 2\nlight, color: [1, 1, 1], position: [0, 5, 0]\n",
    "spot_field": "camera, width: 2, height: 2\nlight, color: [1, 1, 1], radial-a2: 0, radial-a1: 0, "
                  "radial-a0: 1, position: [0, 5, 0], theta: 10\n",
}


@pytest.mark.skipif(not os.path.exists(REF_FRONT), reason="oracle/_ref not built (make ref)")
@pytest.mark.parametrize("name", FIXTURES + sorted(VARIANTS))
def test_parser_matches_reference(name, tmp_path):
    if name in VARIANTS:
        path = str(tmp_path / (name + ".scene"))
        with open(path, "w") as f:
            f.write(VARIANTS[name])
    else:
        path = scene_path(name)
    ref = ctypes.CDLL(REF_FRONT, mode=os.RTLD_LOCAL)
    ours = _parse_with(rc.front_lib(), path)
    theirs = _parse_with(ref, path)
    assert _records(ours) == _records(theirs)


@pytest.mark.skipif(not have_ref(), reason="oracle/_ref not built (make ref)")
@pytest.mark.parametrize("name", sorted(ERRORS))
def test_parse_errors_match_reference(name, tmp_path):
    path = str(tmp_path / (name + ".scene"))
    with open(path, "w") as f:
        f.write(ERRORS[name])
    out = str(tmp_path / "o.ppm")
    a = subprocess.run([CLI, "8", "8", path, out], capture_output=True, text=True, timeout=60)
    b = subprocess.run([os.path.join(REF_DIR, "raytrace_d6"), "8", "8", path, out],
                       capture_output=True, text=True, timeout=60)
    assert (a.returncode, a.stderr) == (b.returncode, b.stderr)
    assert a.returncode == 1 and a.stderr.startswith("Error:")


@pytest.mark.skipif(not os.path.exists(REF_FRONT), reason="oracle/_ref not built (make ref)")
@pytest.mark.parametrize("shape", [(1, 1), (7, 3), (64, 48), (1, 300)])
def test_p3_writer_matches_reference(shape, tmp_path):
    rng = np.random.default_rng(shape[0] * 1000 + shape[1])
    img = rng.integers(0, 256, size=(shape[1], shape[0], 3), dtype=np.uint8)
    img.reshape(-1)[:256] = np.arange(256, dtype=np.uint8)[: img.size]   # every value
    ref = ctypes.CDLL(REF_FRONT, mode=os.RTLD_LOCAL)
    a, b = str(tmp_path / "a.ppm"), str(tmp_path / "b.ppm")
    write_p3(img, a)
    write_p3(img, b, lib=ref)
    assert open(a, "rb").read() == open(b, "rb").read()


def test_libraries_export_header():
    """Every function include/raycast_hip.h declares is exported by one of the libraries."""
    hdr = open(os.path.join(ROOT, "include", "raycast_hip.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    names = set(re.findall(r"\b([a-zA-Z_]\w*)\s*\([^;{]*\)\s*;", hdr))
    names -= {"sizeof", "_Static_assert"}
    hip, front = rc.hip_lib(), rc.front_lib()
    missing = [n for n in sorted(names) if not (hasattr(hip, n) or hasattr(front, n))]
    assert not missing, missing
    assert set(rc.HIP_EXPORTS) <= names and set(rc.FRONT_EXPORTS) <= names


def test_cli_usage_and_open_errors(tmp_path):
    r = subprocess.run([CLI, "1", "2"], capture_output=True, text=True, timeout=60)
    assert (r.returncode, r.stdout) == (0, "Usage: raytrace WIDTH HEIGHT INPUT_SCENE OUTPUT_IMAGE\n")
    r = subprocess.run([CLI, "8", "8", str(tmp_path / "missing.scene"), str(tmp_path / "o.ppm")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1
    assert r.stderr == f"Error: Unable to open the input scene file: {tmp_path / 'missing.scene'}\n"
    r = subprocess.run([CLI, "8", "8", scene_path("simple"), str(tmp_path / "nodir" / "o.ppm")],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 1 and r.stderr.startswith("Error: Unable to open the output image file")


def test_packed_scene_phantom_flags():
    """rc_scene_parity_defined: black phantoms (all fixtures) are defined; a single light with
    color[0]+color[1] < 1 makes the reference read stack garbage."""
    for name in FIXTURES:
        assert rc.Scene.from_file(scene_path(name)).parity_defined()


OPTB = os.path.join(REF_DIR, "raytrace_optb")


@pytest.mark.skipif(not os.path.exists(OPTB), reason="oracle/_ref not built (make ref)")
def test_option_b_links_library(tmp_path):
    """INTEGRATION.md Option B builds: the reference's own main and front end, raycast()
    resolved from libraycast_hip.so (not defined in the binary); the reference's argument
    handling is its own (C/raycast.c:21-24)."""
    nm = subprocess.run(["nm", OPTB], capture_output=True, text=True, check=True).stdout
    assert re.search(r"^\s+U raycast$", nm, flags=re.M), "raycast must come from the library"
    assert re.search(r" T main$", nm, flags=re.M) and re.search(r" T parse_json$", nm, flags=re.M)
    ldd = subprocess.run(["ldd", OPTB], capture_output=True, text=True, check=True).stdout
    assert os.path.join("raytracing-programs_amd", "lib", "libraycast_hip.so") in ldd
    r = subprocess.run([OPTB, "1"], capture_output=True, text=True, timeout=60)
    assert (r.returncode, r.stdout) == (0, "Usage: raytrace WIDTH HEIGHT INPUT_SCENE OUTPUT_IMAGE\n")
    # the reference's main leaves num_lights uninitialised (C/raycast.c:41-44); with the HIP
    # runtime loaded the heap chunk is not zero, and raycast() must still take the lists (it
    # then fails only for want of a GPU, here)
    if not os.path.exists("/dev/kfd"):
        r = subprocess.run([OPTB, "8", "8", scene_path("quadric"), str(tmp_path / "o.ppm")],
                           capture_output=True, text=True, timeout=60)
        assert "could not flatten" not in r.stderr, r.stderr


def test_tuning_api_validates():
    """rc_set_tuning (the explicit replacement for environment knobs) rejects out-of-range
    fields without changing anything and round-trips valid ones; no GPU is touched."""
    base = rc.get_tuning(default=True)
    assert rc.get_tuning() == base
    for bad in (dict(pipe_resolvers=0), dict(pipe_resolvers=5), dict(helpers=65),
                dict(team_blocks=-2), dict(resolve_grid=4), dict(split_shade=1, side=0),
                dict(copy_threads=0), dict(resolve_lds_kb=200), dict(long_len=10), dict(x0=2),
                dict(pipe_order=5), dict(patch_host=3), dict(share_device=2),
                dict(headb_first=-1), dict(pipe_last_whole=2)):
        with pytest.raises(ValueError):
            rc.set_tuning(**bad)
        assert rc.get_tuning() == base, bad
    with rc.tuned(side=0, helpers=1, team_blocks=24):
        t = rc.get_tuning()
        assert (t["side"], t["helpers"], t["team_blocks"]) == (0, 1, 24)
    assert rc.get_tuning() == base
    # the round-5 fields round-trip, and their defaults are the measured schedule
    assert (base["share_device"], base["headb_first"], base["pipe_last_whole"]) == (0, 24, 1)
    with rc.tuned(headb_first=0, share_device=1, pipe_last_whole=0):
        t = rc.get_tuning()
        assert (t["headb_first"], t["share_device"], t["pipe_last_whole"]) == (0, 1, 0)
    # round 6: the early team (measured slower, round 5) is gone from the library
    assert "early_team" not in base and "band_rows" not in base
    assert rc.get_tuning() == base
    with pytest.raises(KeyError):
        rc.set_tuning(no_such_field=1)


def test_binding_loads_one_hip_runtime_from_threads():
    """Threads making their first binding call at once load libraycast_hip.so once, after
    torch: exactly one HIP runtime is mapped (a second one, from /opt/rocm beside torch's,
    corrupts the heap at exit; seen when 8 render threads raced torch's import)."""
    code = (
        "import sys, threading\n"
        "import importlib.util as u\n"
        f"spec = u.spec_from_file_location('rc', {os.path.join(ROOT, 'raytracing-programs_amd', '__init__.py')!r})\n"
        "rc = u.module_from_spec(spec); spec.loader.exec_module(rc)\n"
        "ts = [threading.Thread(target=rc.hip_lib) for _ in range(8)]\n"
        "[t.start() for t in ts]; [t.join() for t in ts]\n"
        "maps = {l.split()[-1] for l in open('/proc/self/maps') if 'libamdhip64' in l}\n"
        "print(len(maps), sorted(maps))\n")
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    assert out.stdout.split()[0] == "1", out.stdout
