"""The reference's data files (Utils/utilities.py:48-101): round trips, the reference's
own error message, and the restricted unpickler refusing anything but arrays."""
import os
import pickle

import numpy as np
import pytest

from conftest import golden
from rti import io as rio


def test_frames_dataset_round_trip(tmp_path):
    d = golden("ptm_perpixel_32x32_N50.npz")
    data = [(d["frames"][i], d["cams"][i]) for i in range(len(d["cams"]))]  # the reference's list of tuples
    path = rio.write_on_file(data, str(tmp_path / "frames_results_coin1"))
    assert path.endswith(".pbz2")
    back = rio.read_from_file(str(tmp_path / "frames_results_coin1"))
    assert len(back) == len(data)
    assert all(np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1]) for a, b in zip(data, back))
    frames, cams = rio.read_frames(str(tmp_path / "frames_results_coin1"))
    assert frames.shape == (50, 32, 32) and frames.dtype == np.uint8 and cams.shape == (50, 3)


def test_tables_round_trip_in_reference_layout(tmp_path):
    d = golden("ptm_perpixel_32x32_N50.npz")
    tables = d["tables"]  # int32 [100, 100, 4, 4], the reference's prepare_images_data output
    path = rio.write_tables(tables, str(tmp_path / "interpolation_results_coin1"))
    assert path.endswith(".pickle")
    with open(path, "rb") as f:
        raw = rio.safe_loads(f.read())
    assert isinstance(raw, list) and isinstance(raw[0], list) and raw[3][7].dtype == np.int32
    assert np.array_equal(rio.read_tables(str(tmp_path / "interpolation_results_coin1")), tables)


def test_missing_file_message_matches_reference(tmp_path):
    with pytest.raises(Exception, match="Storage file not found!"):
        rio.read_from_file(str(tmp_path / "nope"))


class _Evil:
    def __reduce__(self):
        return (os.system, ("echo pwned",))


def test_restricted_unpickler_refuses_code(tmp_path):
    blob = pickle.dumps([np.zeros(3), _Evil()])
    with pytest.raises(pickle.UnpicklingError):
        rio.safe_loads(blob)
    for proto in (2, 4, 5):
        arr = np.arange(12, dtype=np.int32).reshape(3, 4)
        assert np.array_equal(rio.safe_loads(pickle.dumps([(arr, np.float64(2.5))], protocol=proto))[0][0], arr)
