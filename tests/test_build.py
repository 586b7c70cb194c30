"""The tree compiles: the product library is built from this checkout's
sources into a temporary directory (hipcc cross-compiles gfx950 without a
GPU), loads, and exports every symbol the public headers declare. A tree whose
kernels do not compile fails `pytest -m "not gpu"` here, before any GPU run."""
import ctypes
import os
import subprocess
import tempfile

from val_protocol_amd import _build

from .test_abi import _declared_functions


def test_clean_build_into_tmpdir():
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "libval_crc_hip.so")
        _build.build(verbose=False, out=out, build_dir=os.path.join(d, "obj"))
        assert os.path.getsize(out) > 0
        assert _build.is_current(out)
        syms = subprocess.run(["nm", "-D", "--defined-only", out], check=True, capture_output=True,
                              text=True).stdout
        exported = {line.split()[-1] for line in syms.splitlines() if line.strip()}
        missing = sorted(_declared_functions() - exported)
        assert not missing, f"declared but not exported: {missing}"
        ctypes.CDLL(out, mode=ctypes.RTLD_LOCAL)  # loads without a GPU (no compute call)


def test_in_tree_library_is_current():
    """The in-tree .so (what gpurun ships) was built from these sources; crc.lib()
    rebuilds it under a lock otherwise."""
    _build.ensure_built()
    assert _build.is_current()


def test_shipped_library_is_a_product_build():
    """No diagnostic switch is compiled into the in-tree library (those that
    change results cannot even compile without VCRC_DIAG_BUILD)."""
    import val_protocol_amd.crc as vc

    assert vc.build_flags() == ""


def test_wrong_result_switches_need_a_diag_build():
    import shutil

    hipcc = shutil.which("hipcc") or "/opt/rocm/bin/hipcc"
    src = os.path.join(_build.CSRC, "val_crc32_hip.hip")
    for flag in ("-DVCRC_DIAG_NOHASH", "-DVCRC_NO_LDS_FILL", "-DVCRC_REGION_HASHONLY", "-DVCRC_REGION_NOATOMIC"):
        r = subprocess.run([hipcc, "--offload-arch=gfx950", "-std=c++17", "-fsyntax-only", flag, f"-I{_build.INC}",
                            f"-I{_build.CSRC}", src], capture_output=True, text=True)
        assert r.returncode != 0 and "VCRC_DIAG_BUILD" in r.stderr, flag
