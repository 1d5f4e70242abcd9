"""Maps: every lane curve end meets another curve's start (a closed lane graph)
and the product's map builder equals the oracle's restated _load_map/_get_curve."""
import numpy as np
import pytest

from aido1_amd.maps import available_maps, load_map
from conftest import map_rows
from oracle import oracle_c as OC


MAPS = ['loop_empty', 'small_loop', 'zigzag', 'intersections']


@pytest.mark.parametrize('name', MAPS)
def test_lane_graph_closed(name):
    m = load_map(name)
    starts = m.curves[:, 0, :]
    for e in m.curves[:, 3, :]:
        d = np.min(np.linalg.norm(starts - e, axis=1))
        assert d < 1e-9


@pytest.mark.parametrize('name', MAPS)
def test_product_map_equals_oracle_map(name):
    m = load_map(name)
    o = OC.OracleMap(map_rows(name))
    assert np.array_equal(m.kind, o.kind)
    assert np.array_equal(m.curve_start, o.curve_start)
    assert np.array_equal(m.curves, o.curves)
    assert np.array_equal(m.headings, o.headings)


def test_intersection_curve_counts():
    """upstream _get_curve: 2 curves for straight / curve tiles, 6 for a 3-way,
    12 for a 4-way (its 3-curve template at four rotations); a name with '4'
    is a 4-way at angle 2."""
    from aido1_amd.maps import TILE_3WAY_LEFT, TILE_4WAY, parse_rows
    m = load_map('intersections')
    counts = np.diff(m.curve_start)
    assert set(counts[m.kind == TILE_4WAY]) == {12}
    assert set(counts[m.kind == TILE_3WAY_LEFT]) == {6}
    assert set(counts[(m.kind > 0) & (m.kind < TILE_3WAY_LEFT)]) == {2}
    assert set(counts[m.kind <= 0]) == {0}
    four = parse_rows([['4way']])
    assert four.kind[0] == TILE_4WAY and four.orient[0] == 2
    # the four rotations of the template are distinct and each heading block
    # carries the tile-wide Frobenius normalisation
    h = four.headings
    assert abs(np.linalg.norm(h) - 1.0) < 1e-12


def test_available():
    assert {'loop_empty', 'small_loop', 'zigzag'} <= set(available_maps())
