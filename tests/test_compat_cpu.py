"""Host-only parts of the reference-signature adapters (no GPU)."""
import pytest

from conftest import golden
from rti import compat


def test_lookup_mapping_cpu_restatement():
    rows = golden("relight_lookup.npz")["rows"]
    for x, y, h, w, lx, ly, ix, iy in rows:
        got = compat.draw_light_roi_position(int(x), int(y), (int(h), int(w)), to_light_vector=True)
        assert got == (lx, ly) and compat.table_index(got[0]) == ix and compat.table_index(got[1]) == iy


def test_compat_errors_without_gpu():
    import torch

    if torch.cuda.is_available():
        pytest.skip("GPU present")
    with pytest.raises(Exception, match="results are empty"):
        compat.compute_intensities([])
    with pytest.raises(RuntimeError):
        import numpy as np

        z = np.zeros((2, 2, 8), np.float32)
        compat.interpolate_intensities((z, z, z.astype(np.int32)), interpolate_PTM=True)
