"""The reference's C++ test programs against the drop-in header (include/cs/
fm_index.hpp) linked to libcs_fmindex.so: compiled with g++ (CPU, here) and run on
the GPU box."""
import os
import subprocess

import pytest

from conftest import PKG_DIR, ROOT

SRC = os.path.join(ROOT, "tests", "cpp", "facade_tests.cpp")


def _compile(out):
    subprocess.run(["g++", "-std=c++17", "-O2", "-I" + os.path.join(ROOT, "include"), SRC, "-o", out,
                    "-L" + PKG_DIR, "-lcs_fmindex", "-Wl,-rpath," + PKG_DIR], check=True)


def test_facade_compiles_and_links(tmp_path):
    _compile(str(tmp_path / "facade_tests"))


@pytest.mark.gpu
def test_facade_runs_reference_tests(tmp_path):
    exe = str(tmp_path / "facade_tests")
    _compile(exe)
    env = dict(os.environ, FACADE_TMPDIR=str(tmp_path / "idx"))
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300, env=env)
    assert r.returncode == 0, r.stderr
    assert "PASSED" in r.stdout
