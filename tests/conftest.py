import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, 'tests', 'golden')


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a real MI355X (HIP device)')
    config.addinivalue_line('markers', 'slow: long-running CPU test')


def pytest_terminal_summary(terminalreporter):
    """Session total of f16 apsis angles that differ from the reference's by one ulp
    (test_gpu_parity.compare_groups; the per-test bound is ANGLE_MISMATCH_MAX)."""
    gu = sys.modules.get('golden_util')
    ch = getattr(gu, 'CHANGE_TALLY', None)
    if ch:
        n = sum(ch.values())
        terminalreporter.write_line('angle changes vs reference: %d compared, ulp distance histogram %s'
                                    % (n, dict(sorted(ch.items()))))
        per = getattr(gu, 'CHANGE_TALLY_DT', {})
        rel = getattr(gu, 'CHANGE_REL_MAX', {})
        for dt, h in sorted(per.items()):
            terminalreporter.write_line('  %s: %d compared, ulp histogram %s, max relative error %.3g'
                                        % (dt, sum(h.values()), dict(sorted(h.items())),
                                           rel.get(dt, 0.0)))
        _dump('angle_change_ulps.json', dict(
            {str(k): v for k, v in sorted(ch.items())},
            by_dtype={dt: {str(k): v for k, v in sorted(h.items())} for dt, h in per.items()},
            max_rel_error=rel))
    t = getattr(gu, 'ANGLE_TALLY', None)
    if not t or not t['angles']:
        return
    rate = t['mismatch'] / t['angles']
    terminalreporter.write_line('f16 apsis angles vs reference fixtures: %d of %d differ by 1 ulp '
                                '(%.4f %%)' % (t['mismatch'], t['angles'], 100 * rate))
    _dump('angle_mismatch.json', dict(t, rate=rate))


def _dump(name, obj):
    out = os.path.join(ROOT, 'gpurun_out')
    try:
        import json
        os.makedirs(out, exist_ok=True)
        with open(os.path.join(out, name), 'w') as f:
            json.dump(obj, f)
    except OSError:
        pass
