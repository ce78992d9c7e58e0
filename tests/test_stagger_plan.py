"""Host plan of the staggered decoder (janus_amd.pipeline.stagger_plan, CPU): over N slot
sets, every continuing row reads only positions its previous calls wrote (the r04 fault:
a batch-less set continued two chunks ahead onto the -1 token fill), a set holding a
batch continues exactly where it stopped, no call runs past max_length, and batches
complete in order, N calls after they enter — through start-up, steady state and drain."""
import pytest

from janus_amd.pipeline import stagger_plan


def run(n, L, batches):
    S = -(-(L - 1) // n)
    if n * S > L:
        pytest.skip("N does not tile max_length")
    sets, pos, started, k, out, entered = [None] * n, [0] * n, False, 0, [], {}

    def call(batch):
        nonlocal started, k
        offs, jc = stagger_plan(sets, pos, started, k, S, batch is not None)
        f = k % n
        for j in range(n):
            assert offs[j] + S <= L
            if started and not (j == f and batch is not None):
                assert offs[j] <= pos[j], (k, j, offs, pos)
                if sets[j] is not None:
                    assert offs[j] == pos[j]
        if batch is not None:
            assert sets[f] is None           # the fresh set's last batch completed before
        if batch is not None or any(x is not None for x in sets):
            started = True
            for j in range(n):
                pos[j] = offs[j] + S
        if batch is not None:
            sets[f] = {"born": k, "id": batch}
            entered[batch] = k
        if jc is not None:
            b = sets[jc]["id"]
            assert k - entered[b] == n - 1 and pos[jc] >= L - 1  # its rows reached the end
            out.append(b)
            sets[jc] = None
        k += 1

    for b in range(batches):
        call(b)
    while any(x is not None for x in sets):
        call(None)
    return out


@pytest.mark.parametrize("n", [2, 3, 4, 7, 8])
@pytest.mark.parametrize("L", [24, 448])
@pytest.mark.parametrize("batches", [1, 2, 3, 5, 12])
def test_stagger_plan(n, L, batches):
    assert run(n, L, batches) == list(range(batches))


def test_yin_split_start_and_steering():
    """The staggered step's YIN split (JanusPipeline._yin_split, host logic): 7B/8 on the
    decoder side to start when the decoder call leaves room beside it (<= 128 rows), 0 when
    it does not (256-row calls: the decoder side binds); then it follows the previous step's
    side-time gap over twice the per-utterance YIN time, at most 16 per step, within
    [0, B - 1]; a fixed tuning.yin_dec_utts wins."""
    from types import SimpleNamespace

    from janus_amd.pipeline import JanusPipeline, ServingTuning

    class Ev:
        def __init__(self, t):
            self.t = t

        def query(self):
            return True

        def elapsed_time(self, other):
            return other.t - self.t

    fake = SimpleNamespace(tuning=ServingTuning(), YIN_MS_PER_UTT=JanusPipeline.YIN_MS_PER_UTT)
    split = JanusPipeline._yin_split
    assert split(fake, {"n": 2, "R": 64}, 64) == 56
    assert split(fake, {"n": 2, "R": 128}, 64) == 0
    # vocoder side 20 ms longer than the decoder side: move 16 (capped) to the decoder side
    st = {"n": 2, "R": 128, "n_dec": 0, "prev_ev": (Ev(0.0), Ev(300.0), Ev(0.0), Ev(280.0))}
    assert split(fake, st, 64) == 16 and st["n_dec"] == 16
    # decoder side longer: back towards 0, never below
    st["prev_ev"] = (Ev(0.0), Ev(280.0), Ev(0.0), Ev(300.0))
    assert split(fake, st, 64) == 0
    fake.tuning = ServingTuning(yin_dec_utts=70)
    assert split(fake, {"n": 2, "R": 128}, 64) == 63
