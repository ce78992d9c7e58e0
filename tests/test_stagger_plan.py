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
