"""rc_render's in-frame scatter of the mapped colour patch (rc_api.hip scatter_sweep), on the
host alone through the library's test aid rc_debug_scatter_selftest: a writer thread stands in
for phase C, storing this frame's marked entries in shuffled 64-entry batches (each batch in
pieces, as k_dep_chunks does) over entries that still carry an earlier frame's mark.  The
pixmap must come out exactly as expected, and the sweep must end when the frame ends early
(entries never stored) or fails (profiles/r06n_patch_marks.txt, r06p_e2e_tail.txt)."""
import pytest

from helpers import rc


@pytest.mark.parametrize("ndep,seed", [(1, 0), (63, 1), (64, 2), (65, 3), (2047, 4), (2049, 5),
                                       (100_000, 6), (2_804_464, 7)])
def test_scatter_complete_frame(ndep, seed):
    """Every entry stored: every DEP pixel gets its colour, nothing else is touched, and no
    stale entry (an earlier frame's mark) is taken (ndep 2 804 464 = quadric 4096^2 d6)."""
    assert rc.scatter_selftest(ndep, seed) == 0


@pytest.mark.parametrize("skip", [1, 7, 4096])
def test_scatter_frame_that_ends_early(skip):
    """Entries j % skip == 0 never stored, the frame then complete: the sweep ends after one
    more pass and leaves exactly those pixels untouched."""
    assert rc.scatter_selftest(300_000, 11 + skip, skip) == 0


def test_scatter_failed_frame_ends_the_sweep():
    """A frame whose end is reported as a failure while entries are still missing: the sweep
    returns the failure instead of waiting on the entries."""
    assert rc.scatter_selftest(200_000, 3, -5) == -2
    assert rc.scatter_selftest(1, 3, -1) == -2


def test_scatter_rejects_bad_sizes():
    assert rc.scatter_selftest(0, 0) == -1
    assert rc.scatter_selftest((1 << 24) + 1, 0) == -1
