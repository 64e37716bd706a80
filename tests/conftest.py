"""pytest configuration: the `gpu` marker, and an in-tree build before any test runs."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libraycast_hip.so)")


def _built():
    need = ["raytracing-programs_amd/lib/libraycast_hip.so",
            "raytracing-programs_amd/lib/libraycast_front.so",
            "raytracing-programs_amd/bin/raytrace", "oracle/build/liboracle.so"]
    return all(os.path.exists(os.path.join(ROOT, p)) for p in need)


@pytest.fixture(scope="session", autouse=True)
def _build_tree():
    if not _built():
        jobs = os.environ.get("MAX_JOBS", "8")
        subprocess.run(["make", "-j", jobs], cwd=ROOT, check=True, stdout=subprocess.DEVNULL)
    yield
