"""The reference's on-disk formats (Utils/utilities.py:48-101), read safely.

* Frames dataset ``<name>.pbz2`` (analysis.py:434, :460): bz2-compressed cPickle of
  ``list[(V uint8[R, R], camera_position float64[3])]`` — what
  ``FeatureMatcher.extractFeatures`` returns per frame.
* Relight tables ``<name>.pickle`` (analysis.py:475, interactive_relighting.py:95):
  plain pickle of ``list[list[int32[R, R]]]`` indexed ``[ly][lx]``.

Reading uses a restricted unpickler that only rebuilds NumPy arrays, dtypes and
builtin containers/scalars; any other global in the stream raises
``pickle.UnpicklingError`` instead of being imported or called.  Writing
produces files the reference itself can load.
"""
from __future__ import annotations

import bz2
import io
import os
import pickle

import numpy as np

_ALLOWED = {
    ("numpy", "ndarray"), ("numpy", "dtype"),
    ("numpy.core.multiarray", "_reconstruct"), ("numpy._core.multiarray", "_reconstruct"),
    ("numpy.core.multiarray", "scalar"), ("numpy._core.multiarray", "scalar"),
    ("numpy.core.numeric", "_frombuffer"), ("numpy._core.numeric", "_frombuffer"),
    ("builtins", "list"), ("builtins", "tuple"), ("builtins", "dict"), ("builtins", "set"),
    ("builtins", "frozenset"), ("builtins", "bytearray"), ("builtins", "complex"),
    ("_codecs", "encode"),  # protocol-2 bytes payloads of ndarray.__reduce__
}


class _SafeUnpickler(pickle.Unpickler):
    def find_class(self, module, name):
        if (module, name) in _ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f"refusing to load global {module}.{name} from an RTI data file")


def safe_loads(buf):
    """Unpickle ``buf`` allowing only NumPy arrays and builtin containers."""
    return _SafeUnpickler(io.BytesIO(buf)).load()


def _path(filename, compressed):
    return filename + (".pbz2" if compressed else ".pickle")


def write_on_file(data, filename, compressed=True):
    """Utils/utilities.py:48-70: ``<filename>.pbz2`` (bz2 cPickle) or ``<filename>.pickle``."""
    path = _path(filename, compressed)
    if compressed:
        with bz2.BZ2File(path, "wb") as f:
            pickle.dump(data, f)
    else:
        with open(path, "wb") as f:
            pickle.dump(data, f)
    return path


def read_from_file(filename, compressed=True):
    """Utils/utilities.py:73-101 with a restricted unpickler; same missing-file error."""
    path = _path(filename, compressed)
    if not os.path.isfile(path):
        raise Exception("Storage file not found!")
    if compressed:
        with bz2.BZ2File(path, "rb") as f:
            return safe_loads(f.read())
    with open(path, "rb") as f:
        return safe_loads(f.read())


def frames_to_stack(results_frames):
    """list[(V uint8[R,R], cam f64[3])] -> (frames uint8 [N, R, R] light-major, cams f64 [N, 3]).

    The light-major stack is what ``rti.fit(..., cams=cams, mode="perpixel")`` consumes
    (compute_intensities + fit fused on the GPU)."""
    if results_frames is None or len(results_frames) <= 0:
        raise Exception("Error computing intensities: results are empty")
    frames = np.stack([np.asarray(f) for f, _ in results_frames])
    cams = np.stack([np.asarray(c, np.float64).ravel()[:3] for _, c in results_frames])
    return frames, cams


def read_frames(filename, compressed=True):
    """Load a reference frames dataset straight into GPU-ready arrays (frames, cams)."""
    return frames_to_stack(read_from_file(filename, compressed))


def tables_to_reference(tables):
    """int32 [G, G, R, R] -> the reference's ``list[list[int32[R, R]]]`` ([ly][lx])."""
    t = np.asarray(tables)
    return [[np.ascontiguousarray(t[i, j], dtype=np.int32) for j in range(t.shape[1])] for i in range(t.shape[0])]


def write_tables(tables, filename):
    """Write relight tables in the format interactive_relighting.compute() loads (:95)."""
    return write_on_file(tables_to_reference(tables), filename, compressed=False)


def read_tables(filename):
    """Read the reference's relight tables back as an int32 ndarray [G, G, R, R]."""
    return np.asarray(read_from_file(filename, compressed=False), dtype=np.int32)
