"""Maps: every lane curve end meets another curve's start (a closed lane graph)
and the product's map builder equals the oracle's restated _load_map/_get_curve."""
import numpy as np
import pytest

from aido1_amd.maps import available_maps, load_map
from conftest import map_rows
from oracle import oracle_c as OC


@pytest.mark.parametrize('name', ['loop_empty', 'small_loop', 'zigzag'])
def test_lane_graph_closed(name):
    m = load_map(name)
    ends = []
    starts = []
    for t in m.drivable:
        for c in m.curves[t]:
            starts.append(c[0])
            ends.append(c[3])
    starts = np.array(starts)
    for e in ends:
        d = np.min(np.linalg.norm(starts - e, axis=1))
        assert d < 1e-9


@pytest.mark.parametrize('name', ['loop_empty', 'small_loop', 'zigzag'])
def test_product_map_equals_oracle_map(name):
    m = load_map(name)
    o = OC.OracleMap(map_rows(name))
    assert np.array_equal(m.kind, o.kind)
    assert np.array_equal(m.curves, o.curves)
    assert np.array_equal(m.headings, o.headings)


def test_available():
    assert {'loop_empty', 'small_loop', 'zigzag'} <= set(available_maps())
