"""CPU checks of the one-process multi-GPU entry points (include/q2a_encoder.h, q2a_group_*):
the clip-range split is contiguous, near-equal and covers the batch exactly like the torch.distributed path's
q2a.dist.split_batch; without a HIP device q2a_group_open fails with a message instead of falling back."""
import ctypes as C

import pytest

import q2a
from q2a import dist


@pytest.mark.parametrize("n_clips,n_dev", [(512, 8), (64, 1), (7, 3), (3, 8), (0, 4), (1000, 7)])
def test_group_split_is_contiguous_and_matches_dist(n_clips, n_dev):
    rs = q2a.group_split(n_clips, n_dev)
    assert rs == dist.split_batch(n_clips, n_dev)
    assert sum(len(r) for r in rs) == n_clips
    assert [i for r in rs for i in r] == list(range(n_clips))
    assert max(len(r) for r in rs) - min(len(r) for r in rs) <= 1


def test_group_split_rejects_bad_arguments():
    f, c = C.c_int32(), C.c_int32()
    L = q2a.lib()
    for args in ((10, 0, 0), (10, 4, 4), (10, 4, -1), (-1, 4, 0)):
        assert L.q2a_group_split(*args, C.byref(f), C.byref(c)) == -4


def test_group_open_without_device_fails_cleanly(make_model):
    import torch
    if torch.cuda.is_available():
        pytest.skip("a GPU is present")
    path = make_model("tiny", "f16")
    assert q2a.lib().q2a_device_count() == 0
    with pytest.raises(q2a.Q2AError, match="no HIP device"):
        q2a.Group(path)
    with pytest.raises(q2a.Q2AError):
        q2a.Group(path, devices=[0, 0])


def test_group_open_with_needs_an_engine():
    L = q2a.lib()
    assert not L.q2a_group_open_with(None, None, 0)
    assert "invalid arguments" in L.q2a_last_error().decode()
