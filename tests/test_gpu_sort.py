"""The register bitonic sort behind every sorted-segment kernel (wave_dev.h sort2048_reg: A2C update and chain at 256
threads, agent.hip's k_rows_sorted at 512), through toued_sort_keys2048: bit-exact against numpy's sort on the key
forms those kernels build ((row << 11 | sample) and (row << 12 | sample) with 0xFFFFFFFF padding past W*T), on
duplicates, all-equal, sorted and reversed blocks and full-range random words."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

NONE = 0xFFFFFFFF


def _blocks(seed):
    rs = np.random.RandomState(seed)
    out = []
    for shift, TW, D in ((11, 1280, 5409), (12, 1280, 5409), (11, 2048, 70), (12, 64, 3), (11, 0, 10), (11, 1, 2)):
        k = np.full(2048, NONE, np.uint64)
        rows = rs.randint(0, D, TW)
        k[:TW] = (rows.astype(np.uint64) << shift) | np.arange(TW, dtype=np.uint64)
        # the kernels' samples without a row (lifetime-discarded) are NONE in the middle too
        drop = rs.rand(TW) < 0.1
        k[:TW][drop] = NONE
        out.append(k.astype(np.uint32))
    out.append(rs.randint(0, 2 ** 32, 2048, dtype=np.uint64).astype(np.uint32))
    out.append(rs.randint(0, 4, 2048).astype(np.uint32))
    out.append(np.full(2048, 7, np.uint32))
    out.append(np.arange(2048, dtype=np.uint32))
    out.append(np.arange(2048, dtype=np.uint32)[::-1].copy())
    out.append(np.array([0, NONE] * 1024, np.uint32))
    return np.stack(out)


@pytest.mark.parametrize("threads", [256, 512])
def test_sort_keys2048_bitexact(threads):
    from toued import _lib
    keys = _blocks(threads)
    kd = torch.from_numpy(keys.view(np.int32)).cuda()
    od = torch.empty_like(kd)
    _lib.call("toued_sort_keys2048", _lib.ptr(kd), _lib.ptr(od), keys.shape[0], threads, _lib.stream_ptr())
    torch.cuda.synchronize()
    got = od.cpu().numpy().view(np.uint32)
    np.testing.assert_array_equal(got, np.sort(keys, axis=1))


def test_sort_keys2048_many_blocks():
    from toued import _lib
    rs = np.random.RandomState(5)
    keys = rs.randint(0, 2 ** 32, (600, 2048), dtype=np.uint64).astype(np.uint32)
    kd = torch.from_numpy(keys.view(np.int32)).cuda()
    od = torch.empty_like(kd)
    for threads in (256, 512):
        _lib.call("toued_sort_keys2048", _lib.ptr(kd), _lib.ptr(od), keys.shape[0], threads, _lib.stream_ptr())
        torch.cuda.synchronize()
        np.testing.assert_array_equal(od.cpu().numpy().view(np.uint32), np.sort(keys, axis=1))
