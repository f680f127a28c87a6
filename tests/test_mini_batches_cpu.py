"""--num_mini_batches is validated on the GLOBAL agent count, as the reference's mini_batch_vmap reshape does
(util/jax.py:25-41), and each data-parallel rank runs its share as equal chunks no larger than one mini-batch."""
import os
import sys

import pytest

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "to-ued_amd"))
from toued.meta import local_mini_batches  # noqa: E402


@pytest.mark.parametrize("n_local,num_agents,nmb,chunks", [
    (512, 512, 1, 1), (512, 512, 4, 4), (1024, 1024, 2, 2),      # one rank: exactly the reference's split
    (64, 512, 128, 16),                                           # 8 ranks: batch 4 -> 16 chunks of 4
    (64, 512, 1, 1), (64, 512, 8, 1),                             # batch >= the rank's share: one chunk
    (256, 512, 4, 2),                                             # 2 ranks
    (3, 6, 3, 3), (2, 6, 2, 1),
])
def test_local_chunks(n_local, num_agents, nmb, chunks):
    c = local_mini_batches(n_local, num_agents, nmb)
    assert c == chunks
    assert n_local % c == 0 and n_local // c <= num_agents // nmb


def test_global_split_checked():
    with pytest.raises(ValueError, match="num_mini_batches"):
        local_mini_batches(64, 512, 3)
    with pytest.raises(ValueError):
        local_mini_batches(64, 512, 0)


def test_uneven_rank_share_rounds_to_a_divisor():
    # 5 agents on this rank, mini-batch of 2: ceil(5/2) = 3 chunks does not divide 5 -> 5 chunks of 1
    assert local_mini_batches(5, 10, 5) == 5


def test_kernel_range_bounds_a_chunk():
    # one GPU, --num_agents 1024 --num_mini_batches 1: the C2 shape's 1024-agent batch exceeds the GRU kernels'
    # 32-bit operand range (635 agents at K=5, T=20, W=64), so it runs as two equal chunks (numerically a no-op)
    from toued.meta import GRU_MAX_COLUMNS, gru_max_agents
    cap = gru_max_agents(5, 20, 64)
    assert cap == 635 and cap * 5 * 20 * 64 * 264 * 4 < 2 ** 32 and (cap + 1) * 5 * 20 * 64 <= GRU_MAX_COLUMNS + 6400
    assert local_mini_batches(1024, 1024, 1, cap) == 2
    assert local_mini_batches(512, 512, 1, cap) == 1
    assert local_mini_batches(4096, 4096, 1, cap) == 8
    assert local_mini_batches(1024, 1024, 4, cap) == 4      # the requested split is already finer
