"""Wire and disk formats at the edges of the LE path.

Two formats let marker data move between this library and an IBAMR run:

* ``.vertex`` files, the input-deck format of ``IBStandardInitializer``
  (reader: ``src/IB/IBStandardInitializer.cpp:725-790``; sample:
  ``examples/IB/explicit/ex1/curve2d_64.vertex``).  Line 1 holds the vertex count.
  Each following line holds one vertex, NDIM coordinates.  Text after ``!``,
  ``#`` or ``%`` on a line is a comment (``discard_comments``, same file
  :101-123).  Extra tokens after the NDIM coordinates are ignored, as
  ``istringstream >>`` ignores them.  The reader applies
  ``X = length_scale * (X + posn_shift)`` per coordinate (:776).  Errors follow the
  reference's messages: premature end of file, invalid entry, count <= 0.

* The ``LNodeIndex`` stream record (``ibtk/include/ibtk/private/LNodeIndex-inl.h:148-172``):
  three ``int`` (Lagrangian index, global PETSc index, local PETSc index), then
  the periodic offset ``int[NDIM]``, then the periodic displacement
  ``double[NDIM]``.  ``LTransaction::packStream``
  (``ibtk/src/lagrangian/LTransaction.cpp:128-140``) frames a batch as an ``int``
  count, then per item its record and its position ``double[NDIM]``.  IBTK's
  ``FixedSizedStream`` packs these with ``memcpy`` into one buffer, so the bytes
  are host order (little-endian here) with no padding between fields.  SAMRAI's
  ``AbstractStream::sizeofInt/sizeofDouble`` may round each ``pack()`` call up to
  an alignment.  SAMRAI is absent from this image, so that rounding cannot be
  checked; ``align`` exposes it and defaults to 1 (parity unpinned for
  ``align > 1``).

These are host-side formats, so they live in numpy.  The structured arrays map
one-to-one onto ``slab.migrate`` fields: ``X`` is the position, and the index
columns travel as payload.
"""
from __future__ import annotations

import os
from typing import Iterable, Optional, Sequence, Tuple

import numpy as np

__all__ = [
    "read_vertex", "write_vertex",
    "lnode_index_dtype", "lnode_index_stream_size", "pack_lnode_indices", "unpack_lnode_indices",
    "pack_ltransaction", "unpack_ltransaction",
]

_COMMENT_CHARS = "!#%"


def _discard_comments(line: str) -> str:
    """IBStandardInitializer.cpp:101-123: cut at the first '!', then '#', then '%'."""
    for c in _COMMENT_CHARS:
        k = line.find(c)
        if k >= 0:
            line = line[:k]
    return line


def read_vertex(path: str | os.PathLike, ndim: int = 3, length_scale: float = 1.0,
                posn_shift: Optional[Sequence[float]] = None) -> np.ndarray:
    """Read a ``.vertex`` file into an ``(N, ndim)`` float64 array.

    Follows IBStandardInitializer::readVertexFiles (IBStandardInitializer.cpp:725-790).
    Raises ``ValueError`` with the reference's wording on malformed input.
    """
    if ndim not in (2, 3):
        raise ValueError("ndim must be 2 or 3")
    shift = np.zeros(ndim) if posn_shift is None else np.asarray(posn_shift, dtype=np.float64)
    if shift.shape != (ndim,):
        raise ValueError("posn_shift must have ndim entries")
    name = os.fspath(path)
    if not os.path.isfile(name):
        raise FileNotFoundError(f"Cannot find required vertex file: {name}")
    with open(name, "r") as fh:
        first = fh.readline()
        if not first:
            raise ValueError(f"Premature end to input file encountered before line 1 of file {name}")
        tok = _discard_comments(first).split()
        try:
            n = int(tok[0])
        except (IndexError, ValueError):
            raise ValueError(f"Invalid entry in input file encountered on line 1 of file {name}") from None
        if n <= 0:
            raise ValueError(f"Invalid entry in input file encountered on line 1 of file {name}")
        X = np.empty((n, ndim), dtype=np.float64)
        for k in range(n):
            line = fh.readline()
            if not line:
                raise ValueError(f"Premature end to input file encountered before line {k + 2} of file {name}")
            tok = _discard_comments(line).split()
            if len(tok) < ndim:
                raise ValueError(f"Invalid entry in input file encountered on line {k + 2} of file {name}")
            try:
                X[k] = [float(t) for t in tok[:ndim]]
            except ValueError:
                raise ValueError(f"Invalid entry in input file encountered on line {k + 2} of file {name}") from None
    return length_scale * (X + shift)


def write_vertex(path: str | os.PathLike, X: np.ndarray) -> None:
    """Write ``X`` (N, ndim) as a ``.vertex`` file.

    Uses the sample files' style: 17 significant digits in ``%.16e``, so a read
    gives the same doubles back bit for bit.
    """
    X = np.asarray(X, dtype=np.float64)
    if X.ndim != 2 or X.shape[1] not in (2, 3) or X.shape[0] == 0:
        raise ValueError("X must be (N>0, 2|3)")
    with open(os.fspath(path), "w") as fh:
        fh.write(f"{X.shape[0]}\n")
        np.savetxt(fh, X, fmt="%.16e", delimiter=" ")


def _aligned(nbytes: int, align: int) -> int:
    return (nbytes + align - 1) // align * align


def lnode_index_dtype(ndim: int = 3, align: int = 1) -> np.dtype:
    """numpy record dtype of one packed LNodeIndex (LNodeIndex-inl.h:155-163)."""
    if ndim not in (2, 3):
        raise ValueError("ndim must be 2 or 3")
    if align < 1:
        raise ValueError("align must be >= 1")
    names = ["lag", "global_petsc", "local_petsc", "offset", "displacement"]
    formats = ["<i4", "<i4", "<i4", ("<i4", (ndim,)), ("<f8", (ndim,))]
    sizes = [4, 4, 4, 4 * ndim, 8 * ndim]
    offsets, o = [], 0
    for s in sizes:
        offsets.append(o)
        o += _aligned(s, align)
    return np.dtype({"names": names, "formats": formats, "offsets": offsets, "itemsize": o})


def lnode_index_stream_size(ndim: int = 3, align: int = 1) -> int:
    """LNodeIndex::getDataStreamSize (LNodeIndex-inl.h:148-151) at the given alignment."""
    return lnode_index_dtype(ndim, align).itemsize


def _records(lag, global_petsc, local_petsc, offset, displacement, ndim, align):
    lag = np.asarray(lag, dtype=np.int64).reshape(-1)
    n = lag.size
    rec = np.zeros(n, dtype=lnode_index_dtype(ndim, align))
    gp = lag if global_petsc is None else global_petsc
    lp = gp if local_petsc is None else local_petsc
    for name, v in (("lag", lag), ("global_petsc", gp), ("local_petsc", lp)):
        v = np.asarray(v, dtype=np.int64).reshape(-1)
        if v.size != n:
            raise ValueError(f"{name} has {v.size} entries, expected {n}")
        if n and (v.min() < -2**31 or v.max() >= 2**31):
            raise ValueError(f"{name} does not fit in int32")
        rec[name] = v
    if offset is not None:
        rec["offset"] = np.asarray(offset, dtype=np.int32).reshape(n, ndim)
    if displacement is not None:
        rec["displacement"] = np.asarray(displacement, dtype=np.float64).reshape(n, ndim)
    return rec


def pack_lnode_indices(lag, global_petsc=None, local_petsc=None, offset=None, displacement=None,
                       ndim: int = 3, align: int = 1) -> bytes:
    """Pack LNodeIndex records back to back, each as LNodeIndex::packStream writes it.

    ``global_petsc``/``local_petsc`` default to the Lagrangian index; ``offset``
    and ``displacement`` default to zero (a marker with no periodic image).
    """
    return _records(lag, global_petsc, local_petsc, offset, displacement, ndim, align).tobytes()


def unpack_lnode_indices(buf: bytes, ndim: int = 3, align: int = 1) -> np.ndarray:
    """Inverse of :func:`pack_lnode_indices`; returns a structured array."""
    dt = lnode_index_dtype(ndim, align)
    if len(buf) % dt.itemsize:
        raise ValueError(f"buffer of {len(buf)} bytes is not a whole number of {dt.itemsize}-byte records")
    return np.frombuffer(buf, dtype=dt).copy()


def _transaction_dtype(ndim: int, align: int) -> np.dtype:
    idx = lnode_index_dtype(ndim, align)
    return np.dtype({"names": ["index", "posn"], "formats": [idx, ("<f8", (ndim,))],
                     "offsets": [0, idx.itemsize], "itemsize": idx.itemsize + _aligned(8 * ndim, align)})


def pack_ltransaction(records: np.ndarray, posn: np.ndarray, ndim: int = 3, align: int = 1) -> bytes:
    """LTransaction<LNodeIndex>::packStream (LTransaction.cpp:128-140): int count, then per item
    its LNodeIndex record and its position double[NDIM]."""
    records = np.asarray(records)
    posn = np.asarray(posn, dtype=np.float64).reshape(-1, ndim)
    if records.dtype != lnode_index_dtype(ndim, align):
        raise ValueError("records must have lnode_index_dtype(ndim, align)")
    if posn.shape[0] != records.size:
        raise ValueError("one position per record")
    body = np.zeros(records.size, dtype=_transaction_dtype(ndim, align))
    body["index"] = records
    body["posn"] = posn
    head = np.zeros(1, dtype=np.dtype({"names": ["n"], "formats": ["<i4"], "itemsize": _aligned(4, align)}))
    head["n"] = records.size
    return head.tobytes() + body.tobytes()


def unpack_ltransaction(buf: bytes, ndim: int = 3, align: int = 1) -> Tuple[np.ndarray, np.ndarray]:
    """Inverse of :func:`pack_ltransaction`; returns (records, posn (n, ndim))."""
    h = _aligned(4, align)
    if len(buf) < h:
        raise ValueError("buffer shorter than the item count")
    n = int(np.frombuffer(buf[:4], dtype="<i4")[0])
    dt = _transaction_dtype(ndim, align)
    if n < 0 or len(buf) != h + n * dt.itemsize:
        raise ValueError(f"buffer of {len(buf)} bytes does not hold {n} items of {dt.itemsize} bytes")
    body = np.frombuffer(buf[h:], dtype=dt)
    return body["index"].copy(), body["posn"].copy()
