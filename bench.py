"""Headline benchmark: agent-env-steps/sec of the LPG meta-gradient step (BASELINE.json configs[1]).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--env_mode tabular] [--agents_per_gpu 512]
    python -m torch.distributed.run --nnodes=1 --nproc-per-node N --master-addr 127.0.0.1 --master-port P \
        bench.py --gpus N --steps K --warmup W

With --gpus N > 1 and no torchrun environment (WORLD_SIZE unset) the parent starts the N ranks itself
(torch.distributed.run as a child process, before any GPU call in the parent) and exits with their status;
under torchrun WORLD_SIZE must equal --gpus.  Asking for more GPUs than the node has fails loudly.

Workload (C2): env_mode=tabular (the build's defined manual dispatch over the five
LPG tabular levels), num_agents=512 per GPU (weak scaling: 512*N agents
in total), num_mini_batches=1, W=64 workers, T=20, K=5 inner LPG updates,
meta-gradient + Adam, score_function=random level sampling.  A "step" is one
outer iteration of train.py's _meta_train_loop: lpg_meta_grad_train_step then
level_sampler.sample.  value = N_agents_total * W * T * K / seconds per step
(inner-rollout agent-env-steps only; the eval rollout and eval_agent steps are
extra work inside the timed step and are not counted).

Rank 0 prints ONE JSON line.  The dominant kernel's roofline fraction is measured
live with HIP events around its launches on the stream they run on.  The CPU
baseline times the oracle restatement (oracle/, numpy rollout + torch-CPU float32
autograd meta-gradient) on a bounded sample of the same workload.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT / "to-ued_amd"))
sys.path.insert(0, str(ROOT))

import torch  # noqa: E402

MFMA_F32_PEAK_TFLOPS = 157.3       # MI355X_MICROARCH.md: dense f32 MFMA (v_mfma_f32_32x32x2_f32)
MFMA_BF16_PEAK_TFLOPS = 2500.0     # MI355X_MICROARCH.md: dense bf16 MFMA
HBM_PEAK_GBS = 8000.0
# 16-bit MFMA products issued per f32 product (csrc/gru.hip): forward = 16 carry k-steps on scaled fp16 pairs
# (3 products) + 1 input k-step on the exact bf16 triple split (6); backward = the r, z and hn passes on scaled
# fp16 pairs (3 each)
SPLIT_PRODUCTS = {"gru_fwd": (16 * 3 + 6) / 17, "gru_bwd": 3.0}
GRU_FWD_FLOP_PER_ELEM = {5: 406080, 7: 409152}    # per (agent, worker, t)
GRU_BWD_FLOP_PER_ELEM = 2 * 256 * 768              # dh_prev = dG . W_h^T per (k, agent, worker, t)
# algorithmic HBM bytes per element: forward saves h_in, r, z, W_hn h + b_hn (4 x 256 f32; n is
# recomputed by the backward) and reads its inputs/writes its heads (F + 1 + 9 floats); backward reads those four
# saves and the inputs x (F), writes DG (4 x 256), relu(h_out) (256) and DH (9), reading the head cotangents and
# y_hat (1 + 8 + 8) and writing dX3/dX4 (2)
GRU_FWD_BYTES_PER_ELEM = {F: 4 * (4 * 256 + F + 1 + 9) for F in (5, 7)}
GRU_BWD_BYTES_PER_ELEM = {F: 4 * (4 * 256 + F + 5 * 256 + 9 + 17 + 2) for F in (5, 7)}
# with the small weight-gradient products fused (toued_gru_bwd_fused, F <= 6): the four saves and x read, the three
# contraction cotangents DG written (dn_pre, relu(h_out) and DH stay on chip), the head inputs (17 floats) read,
# dX3/dX4 written, one column-exponent byte; the per-workgroup partials (4672 floats per 64 rows x T) are < 0.2 %
GRU_BWD_FUSED_BYTES_PER_ELEM = {F: 4 * (4 * 256 + F + 3 * 256 + 17 + 2) + 1 for F in (5,)}
# main weight-gradient reduction [h_in; x; 1] (256 + F + 1 rows) x [dr; dz; dhn] (768 rows) over M columns: f32-equiv
# FLOP 2 * rows * 768 per column, issued as 3 fp16 products (block-floating-point pairs); algorithmic bytes = both
# operands once (the A rows are re-read by 4 column tiles through L2)
WGRAD_PRODUCTS = 3.0
# the forward's packed fragments a candidate's workgroup reads per step: 16 carry k-steps x 8 unit tiles x 3 gates x
# 2 fp16 pieces + the augmented k-step's 8 unit tiles x 3 gates of 16-byte f32 fragments (FWD_AUG32, the default
# since round 4), 1 KiB each (csrc/gru.hip F6_NFH, F6_A32); the bf16-triple form read 8 x 4 x 3 KiB instead
FWD6_FRAG_BYTES_PER_STEP = (16 * 8 * 3 * 2 + 8 * 3) * 1024
IC_RANDOM_ROWS_GBS = 8600.0        # MI355X_MICROARCH.md: uniformly random rows served by the Infinity Cache
# train rollout: 34 B per agent-env-step (14 written: idx, time, action, reward, done; 20 read: the actor row)
ROLLOUT_BYTES_PER_STEP = 34


def train_rollout_roof():
    """(label, algorithmic bytes per agent-env-step, implementation scratch bytes per agent-env-step) of the train
    rollout as it runs.  The algorithmic figure is SURVEY §8(d)'s 34 B (14 written, the 20-B actor row read) for
    either path; the split path (draws kernel + env chain) also moves its key chain and draws through HBM (u32x4
    written and read back each: 64 B), which is implementation traffic, reported beside it, not counted as work."""
    from toued.rollout import split_rollouts
    if split_rollouts():
        return "toued_rollout_draws + toued_rollout_env (train rollout: threefry draws VALU-bound, env chain " \
               "latency-bound)", ROLLOUT_BYTES_PER_STEP, 16 * 4
    return "k_rollout (train, fused)", ROLLOUT_BYTES_PER_STEP, 0


# device kernel behind each timed region, as rocprofv3 names it (prof_summary.short)
PROFILED_KERNEL = {"gru_fwd": "k_gru_fwd6", "gru_bwd": "k_gru_bwd6n"}


def pmc_traffic(kernel: str):
    """HBM bytes per launch of `kernel` from the newest committed PMC summary (profiles/*/pmc_traffic.json,
    written by tools/profile.sh + tools/prof_summary.py: FETCH_SIZE and WRITE_SIZE passes corrected by the
    calibration factors).  (None, None) when no summary covers the kernel."""
    for d in sorted((ROOT / "profiles").glob("*/pmc_traffic.json"), reverse=True):
        try:
            ks = json.loads(d.read_text())["kernels"]
        except (OSError, ValueError, KeyError):
            continue
        # the kernel by name, or its (single) template instance: "k_wgrad_h3" -> "k_wgrad_h3<8, 2>"
        k = ks.get(kernel) or next((v for n, v in ks.items() if n.startswith(kernel + "<")), None)
        if k:
            return k["hbm_bytes_per_launch"], str(d.relative_to(ROOT))
    return None, None


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--env_mode", default="tabular")
    ap.add_argument("--agents_per_gpu", type=int, default=512)
    ap.add_argument("--lifetime_conditioning", action="store_true")
    ap.add_argument("--no_cpu_baseline", action="store_true")
    ap.add_argument("--workloads", default="c3,c4",
                    help="secondary BASELINE configs measured after the headline at N=1 (comma list of c3, c4; "
                         "'none' to skip): each gets its own value, roofline and cpu_baseline under 'workloads'")
    ap.add_argument("--cpu_agents", type=int, default=0, help="agents in the CPU sample (0 = auto-size to ~15 s)")
    ap.add_argument("--launcher_selftest", action="store_true",
                    help="test hook: run the multi-rank launch, barrier and max-over-ranks timing on gloo/CPU with "
                         "no GPU work, and print the JSON skeleton (tests/test_bench_launch.py)")
    return ap.parse_args()


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(a) -> int:
    """Start --gpus ranks of this script under torch.distributed.run (one process per GPU) and return their exit
    status.  Runs before anything in this process touches the GPU (device_count() does not initialise HIP)."""
    import subprocess
    if not a.launcher_selftest:
        have = torch.cuda.device_count()
        if have < a.gpus:
            raise SystemExit(f"bench.py: --gpus {a.gpus} requested but this node has {have} GPU(s)")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={a.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", str(Path(__file__).resolve()), *sys.argv[1:]]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if a.launcher_selftest:
        env["TOUED_DIST_BACKEND"] = "gloo"
    return subprocess.run(cmd, env=env).returncode


def launcher_selftest(a):
    """Multi-rank plumbing without GPU work: world init, barrier-bracketed timing, MAX over ranks, one line."""
    from toued.dist import init_from_env
    world = init_from_env("gloo")
    world.barrier()
    t0 = time.perf_counter()
    time.sleep(0.01 * (world.rank + 1))
    world.barrier()
    dt = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if world.active:
        import torch.distributed as dist
        dist.all_reduce(dt, op=dist.ReduceOp.MAX)
    # the collectives the step uses, through World: the meta-gradient's all-reduce(SUM) and the sampler's gather
    # of per-agent vectors over the contiguous agent slices (C5: 4096 agents over the ranks)
    lo, hi, n = world.agent_slice(4096)
    s = world.all_reduce_sum(torch.full((4,), float(world.rank + 1)))
    g = world.all_gather_cat(torch.arange(lo, hi, dtype=torch.int32))
    if world.rank == 0:
        print(json.dumps({"metric": "launcher_selftest", "n_gpus": world.size, "ranks_seen": world.size,
                          "max_dt": float(dt), "sum_ranks": float(s[0]), "slice0": [lo, hi, n],
                          "gathered_ok": bool(torch.equal(g, torch.arange(n, dtype=torch.int32)))}), flush=True)
    if world.active:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


def cpu_baseline(env_mode: str, lifetime_conditioning: bool, n_agents: int = 0):
    """Oracle restatement on the host: numpy rollouts + torch-CPU float32 autograd meta-gradient.

    One meta-step (K=5 updates of W=64 x T=20, eval rollout, meta-gradient) for a bounded
    sample of agents; reports agent-env-steps/sec in the same unit as the GPU number."""
    import numpy as np

    from oracle import jaxrand as jr
    from oracle import levels as olv
    from oracle import lpg as olpg
    from oracle import meta as ometa
    from oracle import rollout as oro
    W, T, K = 64, 20, 5
    spec = olv.env_spec(env_mode)
    F = 7 if lifetime_conditioning else 5
    eta = olpg.init_params(0, F).astype(np.float32)

    def run(n):
        keys = jr.split(jr.PRNGKey(0), n)
        p, lt = olv.reset_env_params(keys, env_mode)
        rs = np.random.RandomState(0)
        D = spec.obs_dim
        theta = (rs.randn(n, D, 5) * 0.1).astype(np.float32)
        phi = (rs.randn(n, D, 8) * 0.1).astype(np.float32)
        vc = (rs.randn(n, D, 1) * 0.1).astype(np.float32)
        t0 = time.perf_counter()
        st = oro.batch_reset(spec, jr.split(jr.PRNGKey(1), n), p, W)
        trajs = [[] for _ in range(n)]
        for k in range(K + 1):
            tr, st, _ = oro.batch_rollout(spec, jr.split(jr.PRNGKey(10 + k), n), theta, p, st, T)
            for a in range(n):
                trajs[a].append({kk: v[a] for kk, v in tr.items()})
        agents = [dict(theta=theta[a], phi=phi[a], vcrit=vc[a], step=0, lifetime=int(lt[a]),
                       trajs=trajs[a][:K], eval=trajs[a][K]) for a in range(n)]
        ometa.meta_gradient(eta, agents, ometa.Hypers(lifetime_conditioning=lifetime_conditioning), K,
                            dtype=torch.float32)
        return time.perf_counter() - t0

    if n_agents <= 0:
        t1 = run(1)
        n_agents = int(max(1, min(64, round(15.0 / max(t1, 1e-3)))))
    dt = run(n_agents)
    return {"value": round(n_agents * W * T * K / dt, 1), "unit": "agent-env-steps/sec",
            "cores": torch.get_num_threads(), "kind": "port",
            "sample": f"oracle restatement (numpy rollouts + torch-CPU f32 autograd meta-gradient), one meta-step of "
                      f"{n_agents} agents x W={W} x T={T} x K={K}, env_mode={env_mode}; {dt:.1f} s",
            "cpp_rollout": cpp_rollout_baseline(env_mode)}


def cpp_rollout_baseline(env_mode: str, n_agents: int = 512, target_s: float = 5.0):
    """BASELINE.md §2 variant 2: the C++/OpenMP restatement (oracle/cpu, g++ -O3, bit-exact with the numpy oracle)
    of the rollout + GAE on all host cores: the K train rollouts of N agents x W x T with GAE over each, repeated
    to ~target_s.  agent-env-steps/sec of the rollout part only (no LPG / meta-gradient)."""
    import ctypes
    import numpy as np

    from oracle import cpu
    from oracle import jaxrand as jr
    from oracle import levels as olv
    W, T, K = 64, 20, 5
    spec = olv.env_spec(env_mode)
    D = spec.obs_dim
    p, lt = olv.reset_env_params(jr.split(jr.PRNGKey(0), n_agents), env_mode)
    lev = np.ascontiguousarray(olv.pack_levels(p, lt, spec))
    rs = np.random.RandomState(0)
    theta = (rs.randn(n_agents, D, 5) * 0.5).astype(np.float32)
    vc = (rs.randn(n_agents, D) * 0.1).astype(np.float32)
    from oracle import rollout as oro
    st = oro.batch_reset(spec, jr.split(jr.PRNGKey(1), n_agents), p, W)
    n = n_agents * W
    state = np.zeros((12, n), np.int32)
    state[0], state[1], state[3] = st["time"], st["pos"], st["early_term"]
    state[2] = np.sum(st["obj_existss"] * (1 << np.arange(spec.max_n_objs))[None, :], axis=1)
    state[4:4 + spec.max_n_objs] = st["obj_poss"].T
    idx = np.zeros((n_agents, T + 1, W), np.int32)
    tm = np.zeros_like(idx)
    act = np.zeros((n_agents, T, W), np.uint8)
    rew = np.zeros((n_agents, T, W), np.float32)
    dn = np.zeros_like(act)
    adv = np.zeros((n, T), np.float32)
    tgt = np.zeros_like(adv)
    L = cpu.lib()
    P = lambda a: a.ctypes.data_as(ctypes.c_void_p)
    reps, t0, key = 0, time.perf_counter(), 2
    while True:
        for _ in range(K):
            keys = np.ascontiguousarray(jr.split(jr.PRNGKey(key), n_agents))
            key += 1
            L.toued_cpu_rollout(spec.max_grid_size, spec.max_n_objs, spec.max_n_obj_types, int(spec.tabular), P(lev),
                                P(theta), D, P(keys), P(state), T, W, n_agents, P(idx), P(tm), P(act), P(rew), P(dn),
                                None)
            L.toued_cpu_gae(P(vc), D, P(idx), P(tm), P(rew), P(dn), T, W, n_agents, 0.99, 0.95, P(adv), P(tgt))
        reps += 1
        dt = time.perf_counter() - t0
        if dt >= target_s:
            break
    return {"value": round(reps * K * n * T / dt, 1), "unit": "agent-env-steps/sec", "cores": cpu.threads(),
            "kind": "port", "sample": f"C++/OpenMP restatement (oracle/cpu: rollout + GAE only, no LPG), {reps} x K={K} "
                                      f"rollouts of {n_agents} agents x W={W} x T={T}, env_mode={env_mode}; {dt:.1f} s"}


# ---------------------------------------------------------------------------------------------- C3 / C4 workloads
def _sync_time(fn, n):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    out = None
    for _ in range(n):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n, out


def _hbm_roofline(name, nbytes, mean_ms, note=None, traffic_kernel=None):
    sec = mean_ms * 1e-3
    r = {"bound": "hbm", "kernel": name, "achieved": round(nbytes / sec / 1e9, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(nbytes / sec / 1e9 / HBM_PEAK_GBS, 4), "bytes_per_launch": int(nbytes), "mean_ms": round(mean_ms, 4)}
    if traffic_kernel:
        r["traffic"], r["traffic_source"] = pmc_traffic(traffic_kernel)
    if note:
        r["note"] = note
    return r


def workload_c3(a, cpu: bool):
    """BASELINE C3, GROOVE: --score_function alg_regret --env_mode all_shortlife, 512 agents.  The reference scores
    every agent's level on every meta-step (level_sampler.py:176-181: _compute_algorithmic_regret for all agents,
    the non-terminated scores then masked out), so its meta-step = the LPG meta-gradient step + one regret round
    (a fresh A2C antagonist per agent trained for max_lifetime = 250 updates of W x T, agents/a2c.py:79-125, plus the
    two eval_agent rollouts, level_sampler.py:293-329).  This build scores only terminated agents (the same outputs);
    the regret round is timed with every agent terminated, so t_meta + t_regret is the reference-equivalent step.
    value = inner-rollout agent-env-steps (N W T K of the LPG updates + N U W T of the antagonists) / that time."""
    from toued.env import L_LIFETIME
    from toued.meta import KernelTimers
    from toued.parse_args import parse_args
    from toued.train import Trainer
    N = a.agents_per_gpu
    args = parse_args(["--env_mode", "all_shortlife", "--num_agents", str(N), "--num_mini_batches", "1",
                       "--score_function", "alg_regret"])
    tr = Trainer(args)
    W, T, K = args.env_workers, args.train_rollout_len, args.num_agent_updates
    U = tr.sampler.max_lifetime
    tr.meta_step()                                    # warm: graph capture, code objects
    t_meta, _ = _sync_time(lambda: tr.step_fn(tr.rng, tr.eta, tr.adam, tr.agents), max(1, a.steps))

    def regret_round():
        tr.agents.step = tr.agents.levels[:, L_LIFETIME].clone()     # every agent terminated: all are scored
        tr.buffer, tr.agents = tr.sampler.sample(tr.rng, tr.buffer, tr.agents)
    regret_round()
    t_regret, _ = _sync_time(regret_round, max(1, a.steps))
    # per-kernel launch durations of the antagonists' update chain: one eager round with HIP events (the graph
    # replays the same launches)
    trn = tr.sampler.a2c_trainer()
    trn.timers = KernelTimers()
    trn.timers.enabled = True
    regret_round()
    torch.cuda.synchronize()
    ks = trn.timers.summary()
    trn.timers = None
    D = tr.sampler.obs_dim
    steps_launch = N * W * T
    if "a2c_chain" in ks:
        # toued_a2c_chain: DRAW_CHUNK updates per launch.  Algorithmic bytes per agent-env-step: its draws (16 B),
        # the chosen actor row (20 B) and the V(obs) gather (4 B); the trajectory never leaves LDS
        # launches of 4..32 updates (toued.a2c.chunk_sizes): the per-launch figures are over the mean chunk
        upl = U / ks["a2c_chain"][0]
        chain_ms = ks["a2c_chain"][1]
        dom = _hbm_roofline("k_a2c_chain (A2C antagonist: env chain + fused update, %.2f updates per launch on "
                            "average)" % upl, int(steps_launch * upl * 40), chain_ms,
                            "latency-bound: per update a T-step dependent env chain, then the LDS sort/segment update")
        if "a2c_draws" in ks:
            draws_rf = _hbm_roofline("k_eval_keys + k_eval_draws (state-independent draws of %.2f updates on average)"
                                     % upl, int(steps_launch * upl * 32), ks["a2c_draws"][1], "threefry VALU-bound")
            secondary = {"a2c_chain": dom, "a2c_draws": draws_rf,
                         "per_update_ms": round((chain_ms + ks["a2c_draws"][1]) / upl, 4)}
        else:   # toued_a2c_chain_self: the draws are made inside the chain launch
            dom["kernel"] = ("k_a2c_chain<SELF> (A2C antagonist: env chain + fused update, the next update's draws in "
                             "the idle waves; %.0f updates per launch)" % upl)
            secondary = {"a2c_chain": dom, "per_update_ms": round(chain_ms / upl, 4)}
    else:
        roll_ms, upd_ms = ks["a2c_rollout"][1], ks["a2c_update"][1]
        traj_bytes = N * ((T + 1) * W * 8 + T * W * 6)
        upd_bytes = traj_bytes + N * D * 6 * 4 * 2
        rollout_rf = _hbm_roofline("k_rollout (A2C antagonist train rollout)", steps_launch * ROLLOUT_BYTES_PER_STEP,
                                   roll_ms, "bound in practice by its dependent threefry VALU chain (~12 blocks per step)")
        update_rf = _hbm_roofline("k_a2c_update (fused GAE + actor/critic gradients + clip + SGD, tables in LDS)",
                                  upd_bytes, upd_ms)
        dom = rollout_rf if roll_ms >= upd_ms else update_rf
        secondary = {"a2c_rollout": rollout_rf, "a2c_update": update_rf}
    a2c_steps = N * U * W * T
    meta_steps = N * W * T * K
    t_ref = t_meta + t_regret
    out = {"workload": f"C3 GROOVE alg_regret env_mode=all_shortlife num_agents={N} W={W} T={T} K={K} "
                       f"antagonist updates U={U} (reference-equivalent meta-step: LPG meta-gradient + regret round "
                       f"scoring every agent)",
           "value": round((meta_steps + a2c_steps) / t_ref, 1), "unit": "agent-env-steps/sec",
           "ms_per_step": round(t_ref * 1e3, 3), "meta_updates_per_sec": round(1.0 / t_ref, 3),
           "lpg_meta_step_ms": round(t_meta * 1e3, 3), "regret_round_ms": round(t_regret * 1e3, 3),
           "regret_round_agent_env_steps_per_sec": round(a2c_steps / t_regret, 1),
           "amortized_meta_step_ms": round((t_meta + t_regret * K / U) * 1e3, 3),
           "roofline": dom, "roofline_secondary": secondary,
           "kernels": {k: {"launches": v[0], "mean_ms": round(v[1], 4)} for k, v in ks.items()}}
    out["cpu_baseline"] = c3_cpu_baseline(args, tr.sampler) if cpu else None
    del tr
    torch.cuda.empty_cache()
    return out


def c3_cpu_baseline(args, sampler, target_s: float = 12.0):
    """C3's regret round on the host (C++ rollout/GAE/A2C): the C++/OpenMP restatement (oracle/cpu)
    of n antagonists x U = max_lifetime A2C updates (rollout + GAE + actor/critic update, the A2C update checked
    against the float64 oracle in tests/test_oracle_cpu.py) plus the two eval_agent rollouts per agent (returns
    only, eval length), n sized to ~target_s.  agent-env-steps/sec of the A2C updates, comparable with the GPU's
    regret_round_agent_env_steps_per_sec."""
    import ctypes
    import numpy as np

    from oracle import cpu
    from oracle import jaxrand as jr
    from oracle import levels as olv
    from oracle import rollout as oro
    mode = args.env_mode
    spec = olv.env_spec(mode)
    W, T, D = args.env_workers, args.train_rollout_len, spec.obs_dim
    U, Lr = sampler.max_lifetime, sampler.max_rollout_len
    L = cpu.lib()
    P = lambda x: x.ctypes.data_as(ctypes.c_void_p)

    def run(n, updates):
        p, lt = olv.reset_env_params(jr.split(jr.PRNGKey(0), n), mode)
        lt = np.full_like(lt, 10 ** 6)
        lev = np.ascontiguousarray(olv.pack_levels(p, lt, spec))
        rs = np.random.RandomState(0)
        theta = (rs.randn(n, D, 5) * 0.05).astype(np.float32)
        vc = (rs.randn(n, D) * 0.05).astype(np.float32)
        step = np.zeros(n, np.int32)
        loss = np.zeros((n, 2), np.float32)

        def soa(st, nw):
            s_ = np.zeros((12, n * nw), np.int32)
            s_[0], s_[1], s_[3] = st["time"], st["pos"], st["early_term"]
            s_[2] = np.sum(st["obj_existss"] * (1 << np.arange(spec.max_n_objs))[None, :], axis=1)
            s_[4:4 + spec.max_n_objs] = st["obj_poss"].T
            return s_
        state = soa(oro.batch_reset(spec, jr.split(jr.PRNGKey(1), n), p, W), W)
        idx = np.zeros((n, T + 1, W), np.int32)
        tm = np.zeros_like(idx)
        act = np.zeros((n, T, W), np.uint8)
        rew = np.zeros((n, T, W), np.float32)
        dn = np.zeros_like(act)
        ev_state = soa(oro.batch_reset(spec, jr.split(jr.PRNGKey(2), n), p, 64), 64)
        cum = np.zeros(n * 64, np.float32)
        t0 = time.perf_counter()
        for u in range(updates):
            keys = np.ascontiguousarray(jr.split(jr.PRNGKey(100 + u), n))
            L.toued_cpu_rollout(spec.max_grid_size, spec.max_n_objs, spec.max_n_obj_types, int(spec.tabular), P(lev),
                                P(theta), D, P(keys), P(state), T, W, n, P(idx), P(tm), P(act), P(rew), P(dn), None)
            L.toued_cpu_a2c_update(P(theta), P(vc), P(step), P(lev), D, P(idx), P(tm), P(act), P(rew), P(dn), T, W, n,
                                   0.99, 0.95, 0.01, 40.0, 4.0, 0.5, P(loss))
        for e in range(2):     # eval_agent of the LPG actor and of the trained antagonist: 64 workers x eval length
            keys = np.ascontiguousarray(jr.split(jr.PRNGKey(7 + e), n))
            st_e = ev_state.copy()
            L.toued_cpu_rollout(spec.max_grid_size, spec.max_n_objs, spec.max_n_obj_types, int(spec.tabular), P(lev),
                                P(theta), D, P(keys), P(st_e), Lr, 64, n, None, None, None, None, None, P(cum))
        return time.perf_counter() - t0

    n = 8
    for _ in range(3):       # size n to ~target_s (the parallel efficiency grows with n: re-measure)
        dt = run(n, U)
        if dt >= 0.5 * target_s or n >= 512:
            break
        n = int(max(8, min(512, round(n * target_s / max(dt, 1e-3)))))
    return {"value": round(n * U * W * T / dt, 1), "unit": "agent-env-steps/sec", "cores": cpu.threads(),
            "kind": "port",
            "sample": f"C++/OpenMP restatement (oracle/cpu) of the regret round: {n} antagonists x U={U} A2C updates "
                      f"(rollout + GAE + actor/critic update, W={W}, T={T}) + 2 eval rollouts (64 workers x {Lr} "
                      f"steps) each, env_mode={mode}; {dt:.1f} s"}


def workload_c4(a, cpu: bool):
    """BASELINE C4, TA-LPG: --use_es --lifetime_conditioning --env_mode all_vrandlife, 512 agents -> 1024 OpenES
    candidates (antithetic pairs), each trained with its own LPG for max_lifetime = 250 updates (meta/meta.py:35-37),
    then eval_agent fitness, pair ranks and the OpenES tell (meta/train.py:133-227).  value = candidates x U x W x T
    inner-rollout agent-env-steps per ES step / ES-step time.  The dominant kernel is the per-candidate LPG GRU forward
    (k_gru_fwd6<false>, 16-bit MFMA on the f32-accurate split)."""
    from toued.parse_args import parse_args
    from toued.train import Trainer
    N = a.agents_per_gpu
    args = parse_args(["--env_mode", "all_vrandlife", "--num_agents", str(N), "--num_mini_batches", "1", "--use_es",
                       "--lifetime_conditioning", "--lpg_learning_rate", "0.01"])
    tr = Trainer(args)
    st = tr.step_fn
    W, T, U, C, F = st.W, st.T, st.K, st.C, st.F
    tr.meta_step()
    st.timers.enabled = True
    st.timers.reset()
    n_es = max(1, a.steps // 2)
    t_es, m = _sync_time(tr.meta_step, n_es)
    ks = st.timers.summary()
    st.timers.enabled = False
    R = C * W
    flop = R * T * GRU_FWD_FLOP_PER_ELEM[F]
    g_ms = ks["gru_fwd_multi"][1]
    t_mfma = SPLIT_PRODUCTS["gru_fwd"] * flop / (MFMA_BF16_PEAK_TFLOPS * 1e12)
    # what binds it: every (candidate, step) streams the candidate's whole packed W_h / W_i fragment set (no other
    # workgroup shares it, and 256 resident candidates x 840 KB do not fit the L2s) from the Infinity Cache, against
    # MI355X_MICROARCH.md's 8.6 TB/s (33.5 GB/s per CU) for uniformly random rows served by the Infinity Cache;
    # MFMA (the f32-accurate split's 16-bit products) is the secondary roof
    frag_bytes = C * T * FWD6_FRAG_BYTES_PER_STEP
    sec = g_ms * 1e-3
    rf = {"bound": "infinity-cache", "kernel": "k_gru_fwd6<false> (per-candidate LPG GRU forward)",
          "achieved": round(frag_bytes / sec / 1e9, 1), "peak": IC_RANDOM_ROWS_GBS, "unit": "GB/s",
          "frac": round(frag_bytes / sec / 1e9 / IC_RANDOM_ROWS_GBS, 4), "bytes_per_launch": frag_bytes,
          "mean_ms": round(g_ms, 4),
          "mfma_secondary": {"achieved": round(SPLIT_PRODUCTS["gru_fwd"] * flop / sec / 1e12, 1),
                             "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s (16-bit issued)",
                             "frac": round(t_mfma / sec, 4)},
          "flop_per_launch_f32": flop, "f32_equiv_tflops": round(flop / sec / 1e12, 1)}
    roll_ms = ks["rollout"][1]
    rl, rb, rs_ = train_rollout_roof()
    rollout_rf = _hbm_roofline(rl + " of the candidates", R * T * rb, roll_ms,
                               "bound by its dependent chains (threefry draws, then the env steps), not by bytes")
    rollout_rf["traffic_model"] = R * T * (rb + rs_)
    rollout_rf["traffic_note"] = "algorithmic 34 B + the draws path's key-chain / draws scratch (64 B) per step"
    steps = C * U * W * T
    out = {"workload": f"C4 TA-LPG OpenES env_mode=all_vrandlife lifetime_conditioning num_agents={N} candidates={C} "
                       f"W={W} T={T} updates per candidate U={U}",
           "value": round(steps / t_es, 1), "unit": "agent-env-steps/sec", "ms_per_step": round(t_es * 1e3, 3),
           "meta_updates_per_sec": round(1.0 / t_es, 3), "roofline": rf,
           "roofline_secondary": {"rollout": rollout_rf},
           "kernels": {k: {"launches_per_step": v[0] // n_es, "mean_ms": round(v[1], 4),
                           "total_ms_per_step": round(v[2] / n_es, 3)} for k, v in ks.items()},
           "fitness_mean": float(m["fitness"]["mean"])}
    out["cpu_baseline"] = c4_cpu_baseline(args, tr.sampler) if cpu else None
    del tr
    torch.cuda.empty_cache()
    return out


def c4_cpu_baseline(args, sampler, target_s: float = 12.0):
    """C4 on the host (a subset of candidates, extrapolated and labelled): the oracle restatement
    (numpy rollout + torch-CPU float32 LPG forward and agent update, oracle/meta.py lpg_agent_step) of one candidate's
    lifetime-conditioned LPG updates, as many as fit ~target_s; agent-env-steps/sec of that one candidate's updates.
    The rate per candidate is what a full ES step (1024 candidates x 250 updates) would run at, serially."""
    import numpy as np

    from oracle import jaxrand as jr
    from oracle import levels as olv
    from oracle import lpg as olpg
    from oracle import meta as ometa
    from oracle import rollout as oro
    mode = args.env_mode
    spec = olv.env_spec(mode)
    W, T, D = args.env_workers, args.train_rollout_len, spec.obs_dim
    p, lt = olv.reset_env_params(jr.split(jr.PRNGKey(0), 1), mode)
    eta = torch.from_numpy(olpg.init_params(0, 7).astype(np.float32))
    rs = np.random.RandomState(0)
    theta = torch.from_numpy((rs.randn(D, 5) * 0.1).astype(np.float32))
    phi = torch.from_numpy((rs.randn(D, 8) * 0.1).astype(np.float32))
    hyp = ometa.Hypers(lifetime_conditioning=True)
    st = oro.batch_reset(spec, jr.split(jr.PRNGKey(1), 1), p, W)
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < target_s and n < sampler.max_lifetime:
        tr, st, _ = oro.batch_rollout(spec, jr.split(jr.PRNGKey(10 + n), 1), theta.numpy()[None], p, st, T)
        traj = {k: v[0] for k, v in tr.items()}
        traj["action"] = traj["action"].astype(np.int64)
        traj["done"] = traj["done"].astype(bool)
        th = theta.clone().requires_grad_()
        ph = phi.clone().requires_grad_()
        th, ph, _, _, _ = ometa.lpg_agent_step(th, ph, n, int(lt[0]), eta, traj, hyp)
        theta, phi = th.detach(), ph.detach()
        n += 1
    dt = time.perf_counter() - t0
    return {"value": round(n * W * T / dt, 1), "unit": "agent-env-steps/sec", "cores": torch.get_num_threads(),
            "kind": "port",
            "sample": f"oracle restatement (numpy rollout + torch-CPU f32 lifetime-conditioned LPG forward + agent "
                      f"update) of ONE candidate's first {n} of {sampler.max_lifetime} updates (W={W}, T={T}), "
                      f"env_mode={mode}; {dt:.1f} s; a full ES step is 1024 such candidates x "
                      f"{sampler.max_lifetime} updates (extrapolated: {1024 * sampler.max_lifetime * W * T / (n * W * T / dt):.0f} s)"}


def _event_ms(fn, n):
    """Mean duration (ms) of fn's launches on the current stream, bracketed by HIP events on that stream."""
    fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / n


def micro_gae(n_rows: int = 16384, W: int = 64, T: int = 20):
    """GAE (util/metrics.py:17-38, toued_gae) at the regret round's scale: 32 updates' trajectories of 512 agents
    (16384 x 64 workers x 20 steps = 21 M elements).  SURVEY §8(d): 17 B per element (reward 4 + done 1 + value 4
    read, adv 4 + target 4 written) against 8 TB/s; the value row T (one per worker) is added to the bytes."""
    from toued import _lib
    g = torch.Generator(device="cuda").manual_seed(0)
    v = torch.randn(n_rows, T + 1, W, device="cuda", generator=g)
    r = torch.randn(n_rows, T, W, device="cuda", generator=g)
    d = (torch.rand(n_rows, T, W, device="cuda", generator=g) < 0.05).to(torch.uint8)
    adv, tgt = torch.empty_like(r), torch.empty_like(r)
    gl = float(torch.tensor(0.99 * 0.95, dtype=torch.float32))

    def run():
        _lib.call("toued_gae", n_rows, W, T, _lib.ptr(v), _lib.ptr(r), _lib.ptr(d), 0.99, gl, _lib.ptr(adv),
                  _lib.ptr(tgt), _lib.stream_ptr())
    ms = _event_ms(run, 20)
    elems = n_rows * W * T
    out = _hbm_roofline("k_gae (toued_gae, one lane per worker, reverse scan over T)", elems * 17 + n_rows * W * 4, ms,
                        traffic_kernel="k_gae")
    out["elements"] = elems
    out["elements_per_sec"] = round(elems / (ms * 1e-3), 1)
    return out


def micro_plr(B: int = 4000, N: int = 512, reps: int = 50):
    """The PLR sampler's latency per call at the reference's buffer size (µs per call, not a
    roofline fraction): toued_plr_reset_ids (_reset_lowest_scoring's stable argsort, level_sampler.py:331-353) and
    toued_plr_sample (rank replay + random-new + selection, :203-227, :355-408) on a random buffer, HIP events."""
    from toued import _lib
    g = torch.Generator(device="cuda").manual_seed(1)
    score = torch.rand(B, device="cuda", generator=g)
    active = (torch.rand(B, device="cuda", generator=g) < 0.6).to(torch.uint8)
    new = (torch.rand(B, device="cuda", generator=g) < 0.3).to(torch.uint8)
    ids = torch.empty(N, dtype=torch.int32, device="cuda")
    keys = torch.randint(0, 2 ** 31 - 1, (3, 2), dtype=torch.int32, device="cuda", generator=g)
    chosen, rep, rnd, use = (torch.empty(N, dtype=torch.int32, device="cuda") for _ in range(4))
    st = _lib.stream_ptr()
    t_reset = _event_ms(lambda: _lib.call("toued_plr_reset_ids", B, N, _lib.ptr(score), _lib.ptr(active),
                                          _lib.ptr(new), _lib.ptr(ids), st), reps)
    out = {"buffer_size": B, "num_agents": N, "reset_ids_us": round(t_reset * 1e3, 2)}
    for name, prop in (("sample_rank_us", 0), ("sample_proportional_us", 1)):
        t = _event_ms(lambda: _lib.call("toued_plr_sample", B, N, _lib.ptr(score), _lib.ptr(active), _lib.ptr(new),
                                        _lib.ptr(keys), prop, 1.0, 0.5, _lib.ptr(chosen), _lib.ptr(rep),
                                        _lib.ptr(rnd), _lib.ptr(use), st), reps)
        out[name] = round(t * 1e3, 2)
    out["note"] = "latency-bound single-workgroup kernels (LDS bitonic sort of 8192 keys); µs per call"
    return out


def main():
    a = parse()
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(a))
    if ws != a.gpus:
        raise SystemExit(f"bench.py: --gpus {a.gpus} but WORLD_SIZE={ws}")
    if a.launcher_selftest:
        return launcher_selftest(a)
    from toued.dist import init_from_env
    from toued.parse_args import parse_args
    from toued.train import Trainer
    world = init_from_env()
    n_gpus = world.size
    N_total = a.agents_per_gpu * n_gpus
    cli = ["--env_mode", a.env_mode, "--num_agents", str(N_total), "--num_mini_batches", "1",
           "--score_function", "random"]
    if a.lifetime_conditioning:
        cli.append("--lifetime_conditioning")
    args = parse_args(cli)
    tr = Trainer(args, world)
    step = tr.step_fn
    for _ in range(a.warmup):
        tr.meta_step()

    def timed_pass(with_timers: bool):
        """a.steps meta-steps bracketed by barrier + synchronize, max over ranks.  The headline pass runs with no
        HIP events in the streams (events between launches changed k_wgrad_h3's scheduling once);
        the second pass records the per-kernel events for `kernels` and the roofline."""
        torch.cuda.synchronize()
        world.barrier()
        step.timers.enabled = with_timers
        step.timers.reset()
        torch.cuda.synchronize()
        world.barrier()
        t0 = time.perf_counter()
        for _ in range(a.steps):
            m = tr.meta_step()
        torch.cuda.synchronize()
        world.barrier()
        dt = time.perf_counter() - t0
        step.timers.enabled = False
        tmax = torch.tensor([dt], dtype=torch.float64, device="cuda")
        if world.active:
            import torch.distributed as dist
            dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        return float(tmax), m

    dt, metrics = timed_pass(False)
    dt_timed, _ = timed_pass(True)
    ksum = step.timers.summary()
    W, T, K = args.env_workers, args.train_rollout_len, args.num_agent_updates
    steps_per_meta = N_total * W * T * K
    value = steps_per_meta * a.steps / dt
    F = 7 if a.lifetime_conditioning else 5
    R = a.agents_per_gpu * W
    kern = {}
    for name, (n, mean_ms, tot_ms) in ksum.items():
        kern[name] = {"launches": n, "mean_ms": round(mean_ms, 4), "total_ms_per_step": round(tot_ms / a.steps, 3)}
    # per-launch algorithmic work of the two dominant kernels: f32-equivalent FLOPs and HBM bytes;
    # the roofline bound is whichever roof sets the longer minimum time (bytes / 8 TB/s vs the bf16 MFMA work
    # the f32-accurate split issues / 2.5 PF/s)
    work = {"gru_fwd": (R * T * GRU_FWD_FLOP_PER_ELEM[F], R * T * GRU_FWD_BYTES_PER_ELEM[F]),
            "gru_bwd": (K * R * T * GRU_BWD_FLOP_PER_ELEM,
                        K * R * T * (GRU_BWD_FUSED_BYTES_PER_ELEM[F] if step.gru.fused else GRU_BWD_BYTES_PER_ELEM[F]))}
    cand = [(n, ksum[n][2], ksum[n][1]) for n in work if n in ksum]
    dom, _, mean_ms = max(cand, key=lambda c: c[1])
    flop, nbytes = work[dom]
    t_hbm = nbytes / (HBM_PEAK_GBS * 1e9)
    t_mfma = SPLIT_PRODUCTS[dom] * flop / (MFMA_BF16_PEAK_TFLOPS * 1e12)
    traffic, traffic_src = pmc_traffic(PROFILED_KERNEL[dom])
    sec = mean_ms * 1e-3
    if t_hbm >= t_mfma:
        roofline = {"bound": "hbm", "kernel": dom, "achieved": round(nbytes / sec / 1e9, 1), "peak": HBM_PEAK_GBS,
                    "unit": "GB/s", "frac": round(t_hbm / sec, 4), "bytes_per_launch": nbytes}
    else:
        roofline = {"bound": "mfma", "kernel": dom, "achieved": round(SPLIT_PRODUCTS[dom] * flop / sec / 1e12, 1),
                    "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s (16-bit issued)", "frac": round(t_mfma / sec, 4)}
    roofline.update({"traffic": traffic, "traffic_unit": "bytes/launch", "traffic_source": traffic_src,
                     "mean_ms": round(mean_ms, 4), "min_ms_hbm": round(t_hbm * 1e3, 3),
                     "min_ms_mfma": round(t_mfma * 1e3, 3), "flop_per_launch_f32": flop,
                     "f32_equiv_tflops": round(flop / sec / 1e12, 1), "f32_mfma_peak": MFMA_F32_PEAK_TFLOPS})
    # secondary roofline entries: the weight-gradient reduction (MFMA) and the train rollout (HBM by its bytes; in
    # practice a per-step dependent chain of threefry blocks on the VALU)
    secondary = {}
    M = K * R * T
    if "wgrad_main" in ksum:
        wsec = ksum["wgrad_main"][1] * 1e-3
        wflop = 2.0 * (256 + F + 1) * 768 * M
        wbytes = 4.0 * (256 + F + 1 + 768) * M
        secondary["wgrad"] = {"bound": "mfma", "kernel": "k_wgrad_h3 (+ rowmax, chunk reduce)",
                              "achieved": round(WGRAD_PRODUCTS * wflop / wsec / 1e12, 1),
                              "peak": MFMA_BF16_PEAK_TFLOPS, "unit": "TFLOP/s (16-bit issued)",
                              "frac": round(WGRAD_PRODUCTS * wflop / (MFMA_BF16_PEAK_TFLOPS * 1e12) / wsec, 4),
                              "hbm_gbs": round(wbytes / wsec / 1e9, 1), "mean_ms": round(wsec * 1e3, 4),
                              "traffic": pmc_traffic("k_wgrad_h3")[0]}
    if "rollout" in ksum:
        rsec = ksum["rollout"][1] * 1e-3
        rsteps = R * T
        rl, rb, rs_ = train_rollout_roof()
        secondary["rollout"] = {"bound": "dependent chains (threefry, env steps); hbm by bytes", "kernel": rl,
                                "achieved": round(rsteps * rb / rsec / 1e9, 1),
                                "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                "frac": round(rsteps * rb / rsec / 1e9 / HBM_PEAK_GBS, 4),
                                "bytes_per_launch": rsteps * rb, "traffic_model": rsteps * (rb + rs_),
                                "traffic_note": "algorithmic 34 B + the draws path's key-chain / draws scratch (64 B) "
                                                "per agent-env-step",
                                "agent_env_steps_per_sec": round(rsteps / rsec, 1), "mean_ms": round(rsec * 1e3, 4)}
    out = {
        "metric": "agent-env-steps/sec (inner rollout) at num_agents=512; meta-updates/sec",
        "value": round(value, 1), "unit": "agent-env-steps/sec", "n_gpus": n_gpus, "steps": a.steps,
        "warmup": a.warmup, "ms_per_step": round(dt / a.steps * 1e3, 3), "higher_is_better": True,
        "ms_per_step_timed_pass": round(dt_timed / a.steps * 1e3, 3),
        "timing": "value and ms_per_step from an event-free pass; kernels and roofline from a second pass of the same "
                  "steps with per-kernel HIP events (ms_per_step_timed_pass)",
        "scaling": "weak", "vs_baseline": None, "dtype": "f32",
        "mfma_precision": "f32-class: GRU recurrent products (forward carry, backward gate passes) on power-of-two-"
                          "scaled fp16 pairs (3 fp16 MFMA products, pieces to 2^-22 relative), the weight-gradient "
                          "reduction on block-floating-point fp16 pairs (3 products), the input k-step on the exact "
                          "3-piece bf16 split (6 products), the n gate's input part on f32 MFMA; f32 accumulate",
        "data": "synthetic (procedurally generated levels)",
        "meta_updates_per_sec": round(a.steps / dt, 3),
        "config": {"workload": f"C2 LPG meta-gradient env_mode={a.env_mode} num_agents={N_total} "
                               f"num_mini_batches=1 W={W} T={T} K={K} score_function=random",
                   "num_agents": N_total, "agents_per_gpu": a.agents_per_gpu, "env_workers": W,
                   "train_rollout_len": T, "num_agent_updates": K, "parallelism": f"dp{n_gpus} (agent axis)"},
        "roofline": roofline, "roofline_secondary": secondary, "kernels": kern,
        "metrics": {"lpg_agent_return": float(metrics["lpg_agent_return"].mean()),
                    "lpg_loss": float(metrics["lpg_loss"].mean())},
    }
    if world.rank == 0:
        if not a.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(a.env_mode, a.lifetime_conditioning, a.cpu_agents)
        else:
            out["cpu_baseline"] = None
    if n_gpus == 1:
        out["micro"] = {"gae": micro_gae(), "plr_sampler": micro_plr()}
    wl = [w for w in a.workloads.split(",") if w and w != "none"]
    if wl and n_gpus == 1:
        del tr, step
        torch.cuda.empty_cache()
        out["workloads"] = {}
        for w in wl:
            fn = {"c3": workload_c3, "c4": workload_c4}[w]
            t0w = time.perf_counter()
            out["workloads"][w.upper()] = fn(a, not a.no_cpu_baseline)
            out["workloads"][w.upper()]["wall_s"] = round(time.perf_counter() - t0w, 1)
    if world.rank == 0:
        print(json.dumps(out), flush=True)
    if world.active:
        import torch.distributed as dist
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
