"""Host logic of faster-whisper's temperature fallback (generate_with_fallback) in
janus_amd.services.transcriber, on CPU: the settle rules, the best-of hypothesis choice,
the per-hypothesis noise seeds, and the oracle's noise restatement against a scalar
restatement of decoder.h's hash (the GPU side is tests/test_whisper_gpu.py)."""
import numpy as np

from janus_amd.services import transcriber as tr
from oracle import whisper as ow


def cand(avg, cr=1.0, needs=True, T=0.0, toks=(1, 2)):
    return tr.Candidate(list(toks), avg, 0.0, T, "x", cr, needs)


def test_settle_first_passing_result():
    rs = [cand(-3.0), cand(-0.5, needs=False, T=0.2)]
    assert tr.settle(rs).temperature == 0.2 and tr.settle(rs).avg_logprob == -0.5
    assert tr.settle([cand(-0.2, needs=False)]).temperature == 0.0
    # still running: not every temperature tried and none passed
    assert tr.settle([cand(-3.0), cand(-2.0, T=0.2)]) is None


def test_settle_all_failed_picks_best_avg_under_cr_threshold():
    temps = tr.TEMPERATURES
    rs = [cand(-3.0, T=t) for t in temps]
    rs[2] = cand(-1.5, cr=3.0, T=temps[2])      # best avg but too repetitive
    rs[4] = cand(-2.0, T=temps[4])
    got = tr.settle(rs)
    assert got.avg_logprob == -2.0 and got.temperature == 1.0   # reported at the last T
    # every result above the compression threshold: the best avg of all
    rs = [cand(-3.0 + 0.1 * i, cr=2.5, T=t) for i, t in enumerate(temps)]
    assert tr.settle(rs).avg_logprob == rs[-1].avg_logprob
    # ties: the first (Python max semantics)
    rs = [cand(-2.0, T=t) for t in temps]
    assert tr.settle(rs).tokens == rs[0].tokens


def test_best_hypothesis_score_is_sum_over_length():
    # rows: (tokens, avg_logprob = sum / (len + 1), nsp)
    a = ([1, 2, 3], -4.0 / 4, 0.0)       # sum -4, score -4/3
    b = ([1], -2.0 / 2, 0.0)             # sum -2, score -2
    c = ([1, 2, 3, 4, 5, 6], -7.0 / 7, 0.0)  # sum -7, score -7/6 (best)
    assert tr.best_hypothesis([a, b, c]) is c
    assert tr.best_hypothesis([a, a]) is a
    e = ([], -0.5, 0.0)                  # immediate eot: length 0 counts as 1
    assert tr.best_hypothesis([e, b]) is e


def test_fallback_seed_matches_oracle():
    for key in [(0, 0, 1, 0), (0, 3, 5, 4), (17, 2, 2, 1), (63, 99, 4, 3)]:
        assert tr.fallback_seed(*key) == ow.fallback_seed(*key)
    seeds = {tr.fallback_seed(u, w, t, h) for u in range(4) for w in range(4)
             for t in range(1, 6) for h in range(5)}
    assert len(seeds) == 4 * 4 * 5 * 5


def _mix(h):
    h &= 0xFFFFFFFF
    h ^= h >> 16
    h = (h * 0x85EBCA6B) & 0xFFFFFFFF
    h ^= h >> 13
    h = (h * 0xC2B2AE35) & 0xFFFFFFFF
    return h ^ (h >> 16)


def test_oracle_noise_matches_scalar_hash():
    """oracle.sample_noise (vectorised numpy uint32) = decoder.h's noise_base /
    sample_gumbel restated with Python integers, token by token."""
    V = 4096
    for seed, pos in [(0, 0), (0xDEADBEEF, 447), (12345, 7)]:
        g = ow.sample_noise(seed, pos, V)
        base = _mix(seed ^ _mix((pos * 0x9E3779B9 + 0x7F4A7C15) & 0xFFFFFFFF))
        for t in (0, 1, 255, 4095):
            h = _mix(base ^ ((t * 0x27D4EB2F) & 0xFFFFFFFF))
            u = ((h >> 8) | 1) * 2.0 ** -24
            assert g[t] == -np.log(-np.log(u))
        assert np.isfinite(g).all()
