"""Host logic of the A2C chain path: the chunking of a U-update chain into toued_a2c_chain launches
(toued.a2c.chunk_sizes) and the regret round's sink scatter into the level buffer (toued.plr._scatter_into)."""
import sys
from pathlib import Path

import pytest
import torch

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "to-ued_amd"))


@pytest.mark.parametrize("U", [0, 1, 3, 4, 5, 10, 53, 54, 55, 86, 100, 250, 2500])
def test_chunk_sizes_cover_u(U):
    from toued.a2c import DRAW_CHUNK, DRAW_RAMP, chunk_sizes
    c = chunk_sizes(U)
    assert sum(c) == U
    assert all(1 <= m <= DRAW_CHUNK for m in c)
    assert c == sorted(c)                       # short chunks first, full ones last
    if DRAW_RAMP and U >= sum(DRAW_RAMP) + DRAW_CHUNK:
        assert c[0] == DRAW_RAMP[0] or c[0] < DRAW_RAMP[0]
    if U >= sum(DRAW_RAMP) + DRAW_CHUNK:
        assert c[-1] == DRAW_CHUNK
    # at most one partial chunk beyond the ramp
    assert sum(1 for m in c[len(DRAW_RAMP):] if m != DRAW_CHUNK) <= 1 + len(DRAW_RAMP)


def test_chunk_sizes_ramp_list(monkeypatch):
    from toued.a2c import DRAW_CHUNK, chunk_sizes
    monkeypatch.setenv("TOUED_A2C_RAMP", "4,6,9,14,21")
    c = chunk_sizes(250)
    assert c == [4, 4, 6, 9, 14, 21] + [DRAW_CHUNK] * 6 and sum(c) == 250


def test_chunk_sizes_ramp_off(monkeypatch):
    from toued.a2c import DRAW_CHUNK, chunk_sizes
    monkeypatch.setenv("TOUED_A2C_RAMP", "0")
    c = chunk_sizes(250)
    assert c == sorted(c) and sum(c) == 250 and c.count(DRAW_CHUNK) == 7 and len(c) == 8


def test_scatter_into_sink_drops_writes():
    from toued.plr import _scatter_into
    score = torch.arange(6, dtype=torch.float32)
    term = torch.tensor([True, False, True, False])
    old = torch.tensor([1, 1, 4, 5])
    ids = torch.where(term, old, 6)
    _scatter_into(score, ids, torch.tensor([10.0, 20.0, 30.0, 40.0]))
    assert score.tolist() == [0.0, 10.0, 2.0, 3.0, 30.0, 5.0]
    active = torch.ones(6, dtype=torch.bool)
    _scatter_into(active, ids, False)
    assert active.tolist() == [True, False, True, True, False, True]


def test_self_draws_selection(monkeypatch):
    """toued_a2c_chain_self is the default when the env chain fits one wave and the steps fit its draw flags
    (toued_a2c_chain_self_fits: W <= 64, T <= 64; TOUED_A2C_SELF=0 turns it off).  A long rollout that the chunked
    chain handles (T = 100, W = 16: W*T <= 2048) must fall back to it instead of failing in toued_a2c_chain_self."""
    from toued import _lib
    from toued.a2c import A2CTrainer
    D = 13 * 13 * 2 + 1
    monkeypatch.delenv("TOUED_A2C_SELF", raising=False)
    sd = lambda W, T: A2CTrainer.use_self_draws(None, W, T, D)
    assert sd(64, 20) and not sd(128, 20)
    monkeypatch.setenv("TOUED_A2C_SELF", "1")
    assert sd(64, 20) and sd(32, 20) and sd(32, 64)
    assert not sd(128, 20)
    assert not sd(16, 100) and not sd(16, 65)
    assert _lib.lib().toued_a2c_chain_fits(16, 100, D) == 1      # the chunked chain takes T = 100
    assert _lib.lib().toued_a2c_chain_self_fits(16, 100, D) == 0
    monkeypatch.setenv("TOUED_A2C_SELF", "0")
    assert not sd(64, 20)
