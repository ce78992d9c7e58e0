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


class _FakeEngine:
    """decode_ex stand-in for the sequential fallback: row r's result is a deterministic
    function of its seed (the real decoder's rows are independent of their neighbours and
    keyed by fallback_seed(utt, window, ti, h)), so the sequential and speculative walks see
    the same hypothesis for the same (window, temperature, hypothesis)."""

    class _Out:
        def __init__(self, rows):
            self._rows = rows

        def rows(self):
            return self._rows

    def __init__(self, row_of_seed):
        self.row_of_seed = row_of_seed
        self.calls = 0

    def decode_ex(self, enc, prompts=None, max_length=448, temperature=0.0, seeds=None,
                  enc_index=None, **kw):
        self.calls += 1
        return self._Out([self.row_of_seed(int(s)) for s in seeds])


def test_speculative_walk_matches_sequential():
    """_fallback with every temperature's hypotheses decoded up front (presampled, the
    speculative round) settles every window exactly as the sequential walk: same candidate,
    same temperature, same number of sampled decodes — for windows passing at T = 0, at an
    intermediate temperature, and never."""
    from janus_amd.tokenizer import load_tokenizer
    tk = load_tokenizer()
    temps = tr.TEMPERATURES

    def row_of_seed(s):
        # tokens and avg log-prob from the seed: some hypotheses pass the gates (avg > -1)
        rng = np.random.default_rng(s)
        n = int(rng.integers(3, 12))
        toks = [int(t) for t in rng.integers(0, 5000, n)]
        avg = float(rng.choice([-0.4, -1.6, -2.5, -0.9]))
        return (toks, avg, 0.01)

    # T = 0 rows: window 0 passes, windows 1-4 fail
    first_rows = [([11, 12, 13], -0.3, 0.0)] + [([21, 22], -3.0, 0.0)] * 4
    keys = [(7, 0), (7, 1), (8, 0), (9, 2), (10, 0)]
    prompts = [[1, 2, 3]] * len(keys)
    first = [tr.candidate(tk, t, a, n, 0.0) for t, a, n in first_rows]
    eng = _FakeEngine(row_of_seed)
    seq, nseq = tr._fallback(eng, tk, None, prompts, first, keys, 64, temps, tr.BEST_OF)
    pres = [[[row_of_seed(tr.fallback_seed(k[0], k[1], ti, h)) for h in range(tr.BEST_OF)]
             for ti in range(1, len(temps))] for k in keys]
    spec, nspec = tr._fallback(None, tk, None, prompts, first, keys, 64, temps, tr.BEST_OF,
                               presampled=pres)
    assert nseq == nspec and nseq[0] == 0
    for a, b in zip(seq, spec):
        assert (a.tokens, a.avg_logprob, a.temperature, a.text, a.needs_fallback) == \
            (b.tokens, b.avg_logprob, b.temperature, b.text, b.needs_fallback)
    assert any(0 < n < len(temps) - 1 for n in nseq)   # some settle before the last T
