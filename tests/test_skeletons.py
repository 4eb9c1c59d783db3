"""The skeleton tables that parameterise the bench/test configs equal what the reference's
kinematic classes produce (captured in tests/golden/cov_*.npz by gen_golden.py)."""
import numpy as np
import pytest

from conftest import golden
from skeletondiffusion_amd.skeletons import skeleton


@pytest.mark.parametrize("key,J,ntypes", [("h36m16", 16, 10), ("amass21", 21, 13), ("mano51", 51, 43),
                                          ("freeman17", 17, 9), ("mano52", 52, 44)])
def test_skeleton_tables_match_reference(key, J, ntypes):
    z = golden("cov_" + key)
    names, limbs, adj, types = skeleton(key)
    assert len(names) == J and list(names) == [str(n) for n in z["node_names"]]
    np.testing.assert_array_equal(adj, z["corr"])
    np.testing.assert_array_equal(types, z["node_types"])
    assert types.max() + 1 == ntypes
