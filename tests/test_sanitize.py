"""ASan + UBSan runs of the host C (the CPU restatement must not rely on undefined
behaviour; the front end is the reference's parse/list/writer contract).  `make sanitize`
builds the oracle CLI and a front-end driver (tests/tools/front_check.c) with
-fsanitize=address,undefined and no recovery: any report fails the run.  The sanitized oracle
must still reproduce the reference's md5s; the sanitized front end must parse every fixture
and malformed scene and write the exact P3 bytes.  CPU only."""
import os
import shutil
import subprocess

import numpy as np
import pytest

from helpers import ROOT, file_md5, golden_key, golden_table, rc, scene_path

SAN = os.path.join(ROOT, "build", "sanitize")
FIXTURES = ["simple", "reflection", "quadric", "example2", "example3", "quadric2"]
ENV = dict(os.environ, ASAN_OPTIONS="abort_on_error=0:exitcode=99",
           UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1:exitcode=98")


@pytest.fixture(scope="module")
def built():
    if not shutil.which("gcc"):
        pytest.skip("gcc not available")
    subprocess.run(["make", "-s", "sanitize"], cwd=ROOT, check=True, capture_output=True)
    return SAN


def _clean(r):
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr[-2000:]
    assert "LeakSanitizer" not in r.stderr, r.stderr[-2000:]


@pytest.mark.parametrize("mode", ["parity", "fast"])
def test_oracle_sanitized_goldens(built, mode, tmp_path):
    table = golden_table()
    for name in FIXTURES:
        for d in (0, 4, 6):
            out = str(tmp_path / "o.ppm")
            r = subprocess.run([os.path.join(built, "oracle_raytrace"), "64", "64",
                                scene_path(name), out, str(d), mode],
                               capture_output=True, text=True, timeout=120, env=ENV)
            _clean(r)
            assert r.returncode == 0, r.stderr[-2000:]
            key = golden_key(name, 64, 64, d, mode)
            assert file_md5(out) == table[key]["md5"], key


def test_oracle_sanitized_phantom_and_random(built, tmp_path):
    """Lit phantoms (the light-VLA reconstruction reads) and a ragged size."""
    for name in ("phantom_four", "phantom_two"):
        r = subprocess.run([os.path.join(built, "oracle_raytrace"), "33", "17", scene_path(name),
                            str(tmp_path / "p.ppm"), "6"],
                           capture_output=True, text=True, timeout=120, env=ENV)
        _clean(r)
        assert r.returncode == 0


def test_front_sanitized(built, tmp_path):
    for name in FIXTURES + ["phantom_four", "phantom_two"]:
        out = str(tmp_path / "f.ppm")
        r = subprocess.run([os.path.join(built, "front_check"), scene_path(name), out, "7", "5"],
                           capture_output=True, text=True, timeout=60, env=ENV)
        _clean(r)
        assert r.returncode == 0, r.stderr[-2000:]
        s = rc.Scene.from_file(scene_path(name))
        assert r.stdout.split()[:2] == [str(s.num_shapes), str(s.num_lights)]
        k = np.arange(7 * 5 * 3, dtype=np.int64)
        img = ((k * 7 + k // 3) & 0xFF).astype(np.uint8).reshape(5, 7, 3)
        assert open(out, "rb").read() == rc.encode_p3(img)


@pytest.mark.parametrize("text", [
    "[\n{ type: sphere, color: [1, 0, 0], position: [0, 0, -5] \n]",
    "[\n{ type: camera, width: 2.0, height: 2.0 },\n{ type: cube, position: [0, 0, 0] }\n]",
    "[\n{ type: camera, width: 2.0 height: 2.0 }\n]",
    ""])
def test_front_sanitized_errors(built, tmp_path, text):
    """Malformed input takes the parser's exit(1) paths (C/parse.c messages) without any
    memory error (the reference leaks the lists on those paths too: leak checks off)."""
    path = tmp_path / "bad.scene"
    path.write_text(text)
    env = dict(ENV, ASAN_OPTIONS="detect_leaks=0:exitcode=99")
    r = subprocess.run([os.path.join(built, "front_check"), str(path), str(tmp_path / "o.ppm"),
                        "2", "2"], capture_output=True, text=True, timeout=60, env=env)
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr, r.stderr
    assert r.returncode in (0, 1)
