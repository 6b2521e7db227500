"""Pin the CPU oracle (oracle/orbit_oracle.py) to the reference's own outputs.

Every fixture was produced by importing /root/reference (tools/gen_golden.py); the
oracle must reproduce it bit for bit (NaN == NaN)."""
import numpy as np
import pytest

from golden_util import load, universe, groups, assert_same, assert_groups_equal
from oracle import orbit_oracle as O

BATCH = ['g1_config1', 'g2_overlap_birth_massarray', 'g3_apo_periodic',
         'g4_hubble_catalogue', 'g5_fp32_centre32', 'g5_fp32_centre64',
         'g5_fp32_catalogue32', 'g8_many_small_halos', 'g11_edges']


@pytest.mark.parametrize('name', BATCH)
def test_batch_driver_matches_reference(name):
    fix = load(name)
    u, meta = universe(fix)
    rec = O.track_orbits(u.snapshot_numbers, u.main_branches(), u.regions,
                         u.load_snapshot_data, O.MemoryRecord(), **meta['run'])
    assert rec.attrs['mode'] == str(fix['attr/mode'])
    assert_groups_equal(rec.groups, groups(fix))
    if 'checkpoint/angles' in fix.files:
        assert_same(rec.checkpoint, fix['checkpoint/angles'], 'checkpoint')


@pytest.mark.parametrize('name', ['g1_config1', 'g3_apo_periodic', 'g11_edges'])
def test_resume_matches_reference(name):
    fix = load(name)
    u, meta = universe(fix)
    rec = O.MemoryRecord()
    k = 3
    O.track_orbits(u.snapshot_numbers[:k], u.main_branches()[:k], u.regions,
                   u.load_snapshot_data, rec, **meta['run'])
    O.track_orbits(u.snapshot_numbers, u.main_branches(), u.regions,
                   u.load_snapshot_data, rec, resume=True, **meta['run'])
    assert_groups_equal(rec.groups, groups(fix, 'resume/'))


ONTHEFLY = ['g6_onthefly', 'g6b_onthefly_f32', 'g6c_onthefly_f32_c64', 'g6d_onthefly_empty']


@pytest.mark.parametrize('name', ONTHEFLY)
def test_onthefly_matches_reference(name):
    fix = load(name)
    u, meta = universe(fix)
    for mode in ('pericentric', 'apocentric'):
        got = O.onthefly_track_orbits(meta.get('snapshot', 5), fix['links'], u.regions,
                                      u.load_snapshot_data, mode)
        keys = [k for k in fix.files if k.startswith(mode + '/')]
        assert sorted(k.split('/', 1)[1] for k in keys) == sorted(got), (mode, sorted(got))
        for k in keys:
            d = k.split('/', 1)[1]
            assert_same(np.asarray(got[d]), fix[k], mode + '/' + d)


def test_frame_functions_match_reference():
    fix = load('g7_functions')
    for dt in ('float64', 'float32'):
        base = 'frame_%s' % dt
        x, v, c, m = (fix[base + s] for s in ('/x', '/v', '/c', '/m'))
        for tag, masses, bulk, H0, z in (('mean', 1.0, None, 0.0, 0.0), ('marr', m, None, 72.0, 0.3),
                                         ('cat', 1.0, np.array([0.1, -0.2, 0.3], dtype=dt), 70.0, 1.0)):
            snap = {'coordinates': x, 'velocities': v, 'masses': masses,
                    'box_size': 10.0, 'redshift': z}
            rh, vr, b = O.region_frame(snap, np.array([0, len(x)]), c, bulk,
                                       O.hubble_parameter(z, H0, 0.3, 0.7))
            key = 'frame_%s_%s' % (dt, tag)
            assert_same(rh, fix[key + '/rhat'], key + ' rhat')
            assert_same(vr, fix[key + '/vr'], key + ' vr')
            assert_same(np.asarray(b), fix[key + '/bulk'], key + ' bulk')


def test_compare_and_angles_match_reference():
    fix = load('g7_functions')
    for dt in ('float64', 'float32'):
        base = 'cmp_%s' % dt
        ins = {s: fix[base + '/' + s] for s in
               ('ids', 'ids_prev', 'vr', 'vr_prev', 'rhat', 'rhat_prev', 'angles_prev')}
        for mode in ('pericentric', 'apocentric'):
            key = 'cmp_%s_%s' % (dt, mode)
            d = O.compare_radial_velocities(ins['ids'], ins['ids_prev'], ins['vr'], ins['vr_prev'],
                                            ins['rhat'], ins['rhat_prev'], mode)
            for k, val in d.items():
                want = fix[key + '/out_' + k]
                assert_same(np.asarray(val).astype(want.dtype) if want.dtype.kind == 'i' else val,
                            want, key + ' ' + k)
            a, aa = O.calc_angles(len(ins['ids']), ins['angles_prev'], d)
            assert_same(a, fix[key + '/angles'], key + ' angles')
            assert_same(aa, fix[key + '/apsis_angles'], key + ' apsis_angles')


def test_utils_match_reference():
    fix = load('g7_functions')
    assert_same(O.myin1d(fix['myin1d/a'], fix['myin1d/b']), fix['myin1d/out'], 'myin1d')
    p = fix['recenter/in']
    assert_same(O.recenter_coordinates(p.copy(), 10.0), fix['recenter/scalar'])
    assert_same(O.recenter_coordinates(p.copy(), np.array([10.0, 12.0, 14.0])), fix['recenter/vec3'])
    assert_same(O.recenter_coordinates(p.copy(), np.array([10.0])), fix['recenter/vec1'])
    assert_same(O.recenter_coordinates(p.astype(np.float32), 10.0), fix['recenter/f32_scalar'])


@pytest.mark.parametrize('dt', [np.float64, np.float32])
def test_explicit_reduction_orders_match_numpy(dt):
    """The orders the HIP bulk-velocity kernel implements == numpy's own."""
    rng = np.random.default_rng(11)
    for n in (1, 2, 7, 8, 9, 127, 128, 129, 1000, 8191, 8193, 20001):
        v = (rng.standard_normal((n, 3)) * np.exp(rng.uniform(-4, 4, (n, 3)))).astype(dt)
        assert_same(O.seq_sum_rows(v), np.sum(v, axis=0), 'seq %d' % n)
        a = v[:, 0].copy()
        assert O.pairwise_sum(a) == np.sum(a), n
