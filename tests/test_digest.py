"""librtmi.so carries the digest of the sources it was built from (rt_kernel_source_sha, baked in
by the Makefile), and the binding refuses a library whose digest is not its source tree's: a stale
binary can neither be timed nor profiled under the current sources' name."""
import ctypes
import os
import shutil
import subprocess

import pytest

from raytracingthenextweekcuda_amd import _lib
from raytracingthenextweekcuda_amd.source_digest import digest_files, source_digest
from tests import scenes as S

PKG = os.path.join(S.REPO, "raytracingthenextweekcuda_amd")
CSRC = os.path.join(PKG, "csrc")


def test_in_tree_library_matches_its_sources():
    L = _lib.lib()
    have = _lib.library_digest(L)
    assert len(have) == 16 and have == source_digest(CSRC)
    out = subprocess.run(["make", "-s", "-C", CSRC, "digest"], capture_output=True, text=True, check=True)
    assert out.stdout.strip() == have  # the Makefile and Python compute the same digest


def test_digest_covers_host_sources_header_and_flags():
    names = [n for n, _ in digest_files(CSRC)]
    for f in ("rt_kernel.hip", "rt_kernel.h", "rt_capi.cpp", "rt_scene.cpp", "rt_multi.cpp", "Makefile",
              "include/rtmi.h"):
        assert f in names, f
    assert source_digest(CSRC, "-DRT_CAM_BATCH=16") != source_digest(CSRC)


def _copy_tree(dst):
    """csrc (with its built objects), the digest script and the header, laid out as in the repo."""
    pkg = os.path.join(dst, "pkg")
    shutil.copytree(CSRC, os.path.join(pkg, "csrc"), symlinks=True, copy_function=shutil.copy2,
                    ignore=shutil.ignore_patterns("build_*"))
    shutil.copy2(os.path.join(PKG, "source_digest.py"), pkg)
    os.makedirs(os.path.join(dst, "include"))
    shutil.copy2(os.path.join(S.REPO, "include", "rtmi.h"), os.path.join(dst, "include"))
    return os.path.join(pkg, "csrc"), os.path.join(pkg, "librtmi.so")


def _make(csrc):
    subprocess.run(["make", "-s", "-j4", "-C", csrc, "ARCH=gfx950"], check=True, capture_output=True, timeout=900)


@pytest.mark.timeout(900)
def test_stale_library_is_refused_and_a_rebuild_accepted(tmp_path, monkeypatch):
    if not os.path.isdir(os.path.join(CSRC, "build")):
        pytest.skip("no in-tree build objects to start from")
    monkeypatch.delenv("RTMI_LIB", raising=False)
    csrc, so = _copy_tree(str(tmp_path))
    _make(csrc)  # relinks with the digest of the copied (identical) sources
    fresh = ctypes.CDLL(so)
    assert _lib.check_source_digest(fresh, csrc, so) == source_digest(csrc)

    # a source edit without a rebuild: the library is now stale
    with open(os.path.join(csrc, "rt_scene.cpp"), "a") as fh:
        fh.write("\n// edited after the build\n")
    stale = ctypes.CDLL(so)
    with pytest.raises(_lib.StaleLibraryError, match="stale"):
        _lib.check_source_digest(stale, csrc, so)

    # rebuilding brings the digest back in line (under a new file name: dlopen caches by path)
    _make(csrc)
    so2 = os.path.join(str(tmp_path), "librtmi_rebuilt.so")
    shutil.copy2(so, so2)
    rebuilt = ctypes.CDLL(so2)
    assert _lib.check_source_digest(rebuilt, csrc, so2) == source_digest(csrc) != _lib.library_digest(stale)


def test_experiment_libraries_are_exempt_but_report_their_digest(monkeypatch, tmp_path):
    csrc_copy = os.path.join(str(tmp_path), "pkg", "csrc")
    shutil.copytree(CSRC, csrc_copy, ignore=shutil.ignore_patterns("build*"))
    os.makedirs(os.path.join(str(tmp_path), "include"))
    shutil.copy2(os.path.join(S.REPO, "include", "rtmi.h"), os.path.join(str(tmp_path), "include"))
    with open(os.path.join(csrc_copy, "rt_kernel.h"), "a") as fh:
        fh.write("\n// another tree\n")
    L = _lib.lib()
    with pytest.raises(_lib.StaleLibraryError):
        _lib.check_source_digest(L, csrc_copy)
    monkeypatch.setenv("RTMI_LIB", _lib.LIB_PATH)
    assert _lib.check_source_digest(L, csrc_copy) == _lib.library_digest(L)
