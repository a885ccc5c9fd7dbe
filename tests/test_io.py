"""Wire/disk formats (ibamr_amd.io), CPU only.

Fixtures under tests/golden/vertex/ are data files copied unchanged from the
reference's example input decks:
  curve2d_64.vertex   examples/IB/explicit/ex1 (2-D, no comments)
  sphere3d_32.vertex  examples/IB/explicit/ex2 (3-D, comment on the count line)
  fila_256.vertex     examples/IB/explicit/ex3 (2-D, comments on data lines)
Their known geometry (a sphere of radius 0.5 about the origin, the ex1 ellipse
with semi-axes 0.178571 and 0.35 about (0.5, 0.5)) pins the reader.
"""
import os

import numpy as np
import pytest

from ibamr_amd import io

GOLD = os.path.join(os.path.dirname(__file__), "golden", "vertex")


def test_read_sphere3d_32():
    X = io.read_vertex(os.path.join(GOLD, "sphere3d_32.vertex"))
    assert X.shape == (162, 3)
    r = np.linalg.norm(X, axis=1)
    assert np.abs(r - 0.5).max() < 1e-15


def test_read_curve2d_64():
    X = io.read_vertex(os.path.join(GOLD, "curve2d_64.vertex"), ndim=2)
    assert X.shape == (304, 2)
    assert X[0, 0] == 6.7857142857142860e-01 and X[0, 1] == 0.5
    a, b = 0.5 - X[:, 0].min(), 0.5 - X[:, 1].min()
    assert abs(a - 0.17857142857142855) < 1e-15 and abs(b - 0.35) < 1e-15
    assert np.abs(((X[:, 0] - 0.5) / a) ** 2 + ((X[:, 1] - 0.5) / b) ** 2 - 1).max() < 1e-12


def test_read_comments_per_line():
    X = io.read_vertex(os.path.join(GOLD, "fila_256.vertex"), ndim=2)
    assert X.shape == (201, 2)
    assert X[0].tolist() == [4.5, 14.75]
    assert X[1].tolist() == [4.5002998650, 14.735004501]


def test_scale_and_shift():
    p = os.path.join(GOLD, "sphere3d_32.vertex")
    X = io.read_vertex(p)
    Y = io.read_vertex(p, length_scale=0.25, posn_shift=[2.0, 2.0, 2.0])
    assert np.array_equal(Y, 0.25 * (X + 2.0))


def test_write_read_roundtrip_bitwise(tmp_path):
    rng = np.random.default_rng(3)
    for nd in (2, 3):
        X = rng.standard_normal((1000, nd)) * 10.0 ** rng.integers(-8, 8, (1000, 1))
        p = tmp_path / f"x{nd}.vertex"
        io.write_vertex(p, X)
        assert np.array_equal(io.read_vertex(p, ndim=nd), X)
        assert p.read_text().splitlines()[0] == "1000"


@pytest.mark.parametrize("text, msg", [
    ("", "Premature end"),
    ("0\n", "Invalid entry"),
    ("-3\n", "Invalid entry"),
    ("abc\n", "Invalid entry"),
    ("2\n1 2 3\n", "Premature end to input file encountered before line 3"),
    ("2\n1 2 3\n1 2\n", "Invalid entry in input file encountered on line 3"),
    ("1\n1 x 3\n", "Invalid entry in input file encountered on line 2"),
    ("1\n1 2 # 3\n", "Invalid entry in input file encountered on line 2"),
])
def test_read_errors(tmp_path, text, msg):
    p = tmp_path / "bad.vertex"
    p.write_text(text)
    with pytest.raises(ValueError, match=msg):
        io.read_vertex(p)


def test_missing_file(tmp_path):
    with pytest.raises(FileNotFoundError, match="Cannot find required vertex file"):
        io.read_vertex(tmp_path / "none.vertex")


def test_comment_characters(tmp_path):
    p = tmp_path / "c.vertex"
    p.write_text("2 ! count\n1 2 3 % a\n4 5 6 7 8 # extra tokens are ignored\n")
    assert io.read_vertex(p).tolist() == [[1, 2, 3], [4, 5, 6]]


@pytest.mark.parametrize("ndim", [2, 3])
def test_lnode_index_layout(ndim):
    """Field order and sizes of LNodeIndex::packStream (LNodeIndex-inl.h:155-163) and the
    getDataStreamSize formula (3 + NDIM) * 4 + NDIM * 8 with unpadded packs."""
    assert io.lnode_index_stream_size(ndim) == (3 + ndim) * 4 + ndim * 8
    buf = io.pack_lnode_indices([7], [11], [5], offset=[[1, -1, 0][:ndim]],
                                displacement=[[0.5, -0.25, 2.0][:ndim]], ndim=ndim)
    ints = np.frombuffer(buf[: (3 + ndim) * 4], dtype="<i4")
    dbls = np.frombuffer(buf[(3 + ndim) * 4:], dtype="<f8")
    assert ints.tolist() == [7, 11, 5] + [1, -1, 0][:ndim]
    assert dbls.tolist() == [0.5, -0.25, 2.0][:ndim]


@pytest.mark.parametrize("align", [1, 8])
def test_lnode_pack_roundtrip(align):
    rng = np.random.default_rng(5)
    n = 257
    lag = rng.integers(0, 2**31 - 1, n)
    off = rng.integers(-2, 3, (n, 3))
    disp = rng.standard_normal((n, 3))
    buf = io.pack_lnode_indices(lag, lag + 1, lag % 1000, off, disp, align=align)
    assert len(buf) == n * io.lnode_index_stream_size(3, align)
    r = io.unpack_lnode_indices(buf, align=align)
    assert np.array_equal(r["lag"], lag) and np.array_equal(r["global_petsc"], lag + 1)
    assert np.array_equal(r["local_petsc"], lag % 1000)
    assert np.array_equal(r["offset"], off) and np.array_equal(r["displacement"], disp)
    with pytest.raises(ValueError):
        io.unpack_lnode_indices(buf[:-1], align=align)


def test_lnode_defaults_and_range():
    r = io.unpack_lnode_indices(io.pack_lnode_indices([3, 4]))
    assert r["global_petsc"].tolist() == [3, 4] and r["local_petsc"].tolist() == [3, 4]
    assert not r["offset"].any() and not r["displacement"].any()
    with pytest.raises(ValueError, match="int32"):
        io.pack_lnode_indices([2**31])


@pytest.mark.parametrize("ndim", [2, 3])
def test_ltransaction_roundtrip(ndim):
    """LTransaction::packStream framing (LTransaction.cpp:128-140): int count, then
    (record, posn double[NDIM]) per item."""
    rng = np.random.default_rng(ndim)
    n = 40
    rec = io.unpack_lnode_indices(io.pack_lnode_indices(np.arange(n), ndim=ndim), ndim=ndim)
    X = rng.random((n, ndim))
    buf = io.pack_ltransaction(rec, X, ndim=ndim)
    item = io.lnode_index_stream_size(ndim) + 8 * ndim
    assert len(buf) == 4 + n * item
    assert np.frombuffer(buf[:4], "<i4")[0] == n
    assert np.frombuffer(buf[4 + item - 8 * ndim: 4 + item], "<f8").tolist() == X[0].tolist()
    r2, X2 = io.unpack_ltransaction(buf, ndim=ndim)
    assert np.array_equal(r2, rec) and np.array_equal(X2, X)
    r0, X0 = io.unpack_ltransaction(io.pack_ltransaction(rec[:0], X[:0], ndim=ndim), ndim=ndim)
    assert r0.size == 0 and X0.shape == (0, ndim)
    with pytest.raises(ValueError):
        io.unpack_ltransaction(buf[:-8], ndim=ndim)
