"""GPU tests of the reference's debug hooks (util/jax.py:5-17) and of the device error word.

* toued_nonfinite_count (--debug_nans' per-stage reduction) against torch.isfinite at several sizes;
* --debug_nans: a NaN poisoned into eta raises FloatingPointError at the first stage it reaches (the GRU states or
  the LPG outputs of inner update 0), a clean run raises nothing and matches the run without the flag bit for bit;
* --debug: the meta-step with a synchronise + error check after every ABI call equals the normal one;
* toued_a2c_chain_self's bounded flag wait: with the key wave's publish of one step suppressed
  (TOUED_TEST_A2C_SKIP_PUBLISH, tests only) the expired wait is reported as ToUEDError through
  toued_device_error_check (agents/a2c.py:79-125 is the scan it runs), and a normal run reports nothing.
"""
import pytest
import torch

from oracle import jaxrand as jr

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True)
def _reset_debug():
    yield
    from toued import debug
    debug.configure(False, False)


@pytest.mark.parametrize("n", [1, 257, 100_000, 3_000_001])
def test_nonfinite_count_matches_torch(n):
    from toued import _lib
    g = torch.Generator(device="cuda").manual_seed(n)
    x = torch.randn(n, device="cuda", generator=g)
    idx = torch.randint(0, n, (min(n, 50),), device="cuda", generator=g)
    x[idx[: len(idx) // 2]] = float("nan")
    x[idx[len(idx) // 2:]] = float("-inf") if n % 2 else float("inf")
    x[0] = 3.0e38    # finite extremes are not counted
    out = torch.zeros(2, dtype=torch.int32, device="cuda")
    _lib.call("toued_nonfinite_count", _lib.ptr(x), n, _lib.ptr(out) + 4, _lib.stream_ptr())
    _lib.call("toued_nonfinite_count", _lib.ptr(x), n, _lib.ptr(out) + 4, _lib.stream_ptr())
    assert out.cpu().tolist() == [0, 2 * int((~torch.isfinite(x)).sum())]


def test_nonfinite_count_2d_column_block():
    from toued import _lib
    x = torch.randn(40, 1000, device="cuda")
    x[3, 110] = float("nan")    # inside the block (columns 100 .. 799)
    x[7, 600] = float("inf")    # inside
    x[5, 999] = float("nan")    # outside
    x[6, 50] = float("nan")     # outside
    blk = x[:, 100:800]
    out = torch.zeros(1, dtype=torch.int32, device="cuda")
    _lib.call("toued_nonfinite_count_2d", blk.data_ptr(), 40, 700, 1000, _lib.ptr(out), _lib.stream_ptr())
    assert int(out) == int((~torch.isfinite(blk)).sum()) == 2


def _trainer(extra=()):
    from toued.parse_args import parse_args
    from toued.train import Trainer
    args = parse_args(["--env_mode", "dense", "--num_agents", "4", "--num_mini_batches", "1",
                       "--num_agent_updates", "2", "--seed", "3", *extra])
    return Trainer(args)


@pytest.mark.parametrize("param,stage", [("hr_w", "lpg_gru_states"), ("pi_w", "lpg_outputs")])
def test_debug_nans_poisoned_eta_raises_at_first_stage(param, stage):
    """A NaN in a recurrent weight (or in the embedding MLP that feeds the GRU inputs) first shows in the GRU states
    of inner update 0 (the heads read relu(h) = max(h, 0), which maps it to 0 on the device); one in a head weight in
    the LPG outputs."""
    tr = _trainer(["--debug_nans"])
    off = tr.step_fn.lay.offsets[param]
    tr.eta[off + 5] = float("nan")
    with pytest.raises(FloatingPointError, match=f"stage '{stage}'"):
        tr.meta_step()


def test_debug_flags_clean_run_is_bit_identical():
    """--debug_nans and --debug on a clean run: no raise, and the same eta / agents as without them."""
    runs = []
    for extra in ((), ("--debug_nans",), ("--debug", "--debug_nans")):
        tr = _trainer(extra)
        for _ in range(2):
            tr.meta_step()
        tr.finish()
        torch.cuda.synchronize()
        runs.append((tr.eta.clone(), tr.agents.theta.clone(), tr.agents.levels.clone()))
    for r in runs[1:]:
        for a, b in zip(runs[0], r):
            assert torch.equal(a, b)


def test_a2c_chain_self_expired_wait_is_reported(monkeypatch):
    from test_gpu_plr import _a2c_setup, _ahyp, dk
    from toued import _lib
    from toued.a2c import A2CHyperparams, A2CTrainer
    monkeypatch.setenv("TOUED_A2C_SELF", "1")
    mode, N, W, T, U = "dense", 2, 64, 20, 3
    ro, levels, p, lt, theta, vcrit, state, D = _a2c_setup(mode, N, W, T, seed=5)
    rng = dk(jr.split(jr.PRNGKey(11), N))

    def run():
        th, vc, st = theta.clone(), vcrit.clone(), state.clone()
        step = torch.zeros(N, dtype=torch.int32, device="cuda")
        tr = A2CTrainer(ro, A2CHyperparams(), _ahyp(mode), use_graph=False)
        assert tr.use_self_draws(W, T, D)
        tr.train(rng, th, vc, step, levels, st, U)
        return th

    _lib.check_device_errors(wait=True)          # a clean word to start from
    good = run()
    _lib.check_device_errors(wait=True)
    monkeypatch.setenv("TOUED_TEST_A2C_SKIP_PUBLISH", "1")
    bad = run()
    with pytest.raises(_lib.ToUEDError, match="draw wave's wait for the key wave's flag expired"):
        _lib.check_device_errors(wait=True)
    # the word is cleared by the report (here the late keys had landed before the wave read them, so the result is
    # still right: the error reports the expired wait itself, whatever it then read)
    _lib.check_device_errors(wait=True)
    del bad
    monkeypatch.delenv("TOUED_TEST_A2C_SKIP_PUBLISH")
    again = run()
    _lib.check_device_errors(wait=True)
    assert torch.equal(good, again)
