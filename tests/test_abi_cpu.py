"""CPU tests of the C-ABI library: it loads and exports every symbol include/*.h declares.

No compute call is made here (no GPU in this container); the GPU tests exercise them.
"""
import ctypes
import re
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def declared_functions():
    names = set()
    for h in (ROOT / "include").glob("*.h"):  # the C-ABI headers (the C++ facade is checked below)
        text = h.read_text()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        text = re.sub(r"\btypedef\b[^;]*;", "", text)  # function-pointer types are not functions
        for m in re.finditer(r"^\s*(?:const\s+)?[A-Za-z_][\w\s\*]*?\b(\w+)\s*\(", text, flags=re.M):
            name = m.group(1)
            if name in ("if", "while", "for", "return", "sizeof", "defined"):
                continue
            names.add(name)
    return sorted(names)


@pytest.fixture(scope="module")
def lib():
    from ibamr_amd import _lib
    if not _lib.LIB_PATH.exists():
        from ibamr_amd import build
        build.build()
    return _lib.load()


def test_headers_declare_the_abi():
    names = declared_functions()
    assert "ibtk_le_interp" in names and "ibtk_le_spread" in names
    assert "lagrangian_ib_4_interp3d_" in names and "lagrangian_ib_6_spread2d_" in names
    assert len([n for n in names if n.startswith("lagrangian_")]) == 32


def test_library_exports_every_declared_symbol(lib):
    missing = [n for n in declared_functions() if not hasattr(lib, n)]
    assert not missing, f"not exported: {missing}"


def test_host_only_helpers(lib):
    from ibamr_amd import _lib
    assert _lib.kernel_id("IB_4") == 5
    assert lib.ibtk_le_stencil_size(_lib.kernel_id("IB_6")) == 6
    # LEInteractor::getMinimumGhostWidth: floor(stencil/2)+1
    expect = {"PIECEWISE_CONSTANT": 1, "DISCONTINUOUS_LINEAR": 2, "PIECEWISE_LINEAR": 2, "PIECEWISE_CUBIC": 3,
              "IB_3": 3, "IB_4": 3, "IB_4_W8": 5, "IB_6": 4, "BSPLINE_4": 3}
    for k, g in expect.items():
        assert lib.ibtk_le_min_ghost_width(_lib.kernel_id(k)) == g
    assert lib.ibtk_le_kernel_from_name(b"USER_DEFINED") == 9  # ibtk_le_user_interp / _spread
    assert lib.ibtk_le_stencil_size(9) == 4 and lib.ibtk_le_min_ghost_width(9) == 3  # ib4_kernel_fcn, 4
    with pytest.raises(_lib.IBTKLEError):
        _lib.kernel_id("NOPE")


def test_no_oracle_in_product_path():
    """The product package never imports the oracle (it is test infrastructure)."""
    pat = re.compile(r"(import\s+oracle|from\s+oracle|le_oracle|libleoracle|ora_interp|ora_spread)")
    for p in (ROOT / "ibamr_amd").rglob("*"):
        if p.suffix in (".py", ".cpp", ".hip", ".h"):
            assert not pat.search(p.read_text()), p


def test_cpp_facade_methods_exported(lib):
    """The C++ LEInteractor facade (include/ibtk_le/LEInteractor.h) is compiled into the library."""
    import shutil
    import subprocess
    nm = shutil.which("nm")
    if nm is None:
        pytest.skip("nm not available")
    from ibamr_amd import _lib
    out = subprocess.run([nm, "-DC", str(_lib.LIB_PATH)], capture_output=True, text=True).stdout
    hdr = (ROOT / "include" / "ibtk_le" / "LEInteractor.h").read_text()
    methods = sorted(set(re.findall(r"static\s+\w+\s+(\w+)\(", hdr)))
    assert {"interpolate", "spread", "getStencilSize", "getMinimumGhostWidth"} <= set(methods)
    for m in methods:
        assert f"IBTK::LEInteractor::{m}(" in out, m
    # the reference's 16 interpolate and 16 spread overloads (LEInteractor.h:146-993):
    # {LData + index set, raw + index set, std::vector, raw with sizes} x {Cell, Node,
    # Side, Edge}, overloaded by data type
    for m in ("interpolate", "spread"):
        sigs = {ln for ln in out.splitlines() if f"IBTK::LEInteractor::{m}(" in ln}
        assert len(sigs) == 16, (m, len(sigs))
        # Cell / Node / Side / Edge = ScalarDataView<0>, <1>, VectorDataView<0>, <1>
        for view in ("ScalarDataView<0>", "ScalarDataView<1>", "VectorDataView<0>", "VectorDataView<1>"):
            assert sum(1 for ln in sigs if view in ln) == 4, (m, view)


def test_argument_errors_before_any_device_call(lib):
    """Entry points reject bad arguments with IBTK_LE_ERR_ARG (4) before touching a
    device, as the reference's TBOX_ERROR checks come before any work."""
    import ctypes
    from ibamr_amd import _lib
    g = _lib.PatchGeom.make([0, 0, 0], [7, 7, 7], [2, 2, 2], [0.1] * 3, [0.0] * 3, [0.8] * 3)
    n = ctypes.c_int(0)
    assert lib.ibtk_le_phys_bdry_side(None, ctypes.byref(g), None, None, None, None, None, 1) == 4
    assert lib.ibtk_le_local_numbering(None, ctypes.byref(g), None, 10, None, ctypes.byref(n)) == 4
    assert lib.ibtk_le_position_update(None, 0, 10, 0.1, None, None, None, None) == 4
    msg = lib.ibtk_le_last_error().decode()
    assert msg, "the last error carries a message"
