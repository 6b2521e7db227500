"""Pin the §8(f) oracle (oracle/post_oracle.py: collate_apsides,
save_final_apsis_counts, get_central_particle_ids, find_main_progenitors) to the
reference's own outputs (g9_collate, g10_progenitors), bit for bit."""
import numpy as np
import pytest

from golden_util import assert_same
from post_golden import collate_runs, central_cases, mainprog_cases
from oracle import post_oracle as PO

RUNS = collate_runs()


@pytest.mark.parametrize('run', RUNS, ids=['%s-%s' % r[:2] for r in RUNS])
def test_collate_oracle_matches_reference(run):
    case, tag, groups, attrs, kw, fkw, want = run
    got = PO.collate_apsides(groups, attrs, **kw)
    if fkw is not None:
        fin = PO.save_final_apsis_counts(got, attrs['mode'], **fkw)
        t = '{}er_counts_final'.format(attrs['mode'][:-3])
        for g, v in fin.items():
            got[g][t] = v
    assert sorted(got) == sorted(want)
    for g in want:
        assert list(got[g]) == list(want[g]), (g, list(got[g]), list(want[g]))
        for d in want[g]:
            assert_same(got[g][d], want[g][d], '%s/%s/%s' % (tag, g, d))


@pytest.mark.parametrize('case', central_cases(), ids=lambda c: c[0])
def test_central_ids_oracle_matches_reference(case):
    name, snap, pos, n, want_ids, want_off = case
    ids, off = PO.get_central_particle_ids(snap, pos, n=n)
    assert_same(ids, want_ids, name + '/ids')
    assert_same(off, want_off, name + '/offsets')


@pytest.mark.parametrize('case', mainprog_cases(), ids=lambda c: c[0])
def test_main_progenitors_oracle_matches_reference(case):
    name, hp, ho, tp, to, want = case
    got = PO.find_main_progenitors(hp, ho, tp, to)
    assert np.array_equal(np.array([int(v) for v in got]), want), name


def test_collate_rejects_unprocessed_halo():
    case, tag, groups, attrs, kw, fkw, want = RUNS[0]
    with pytest.raises(ValueError):
        PO.collate_apsides(groups, attrs, halo_ids=np.array([10 ** 9]))
