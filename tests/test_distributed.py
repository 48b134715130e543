"""CPU tier: the multi-GPU path (trial sharding + one all-reduce of the NMSE/LLF
accumulators) exercised with the gloo backend at world sizes 2 and 4.  Per-trial
NMSE comes from the CPU oracle here (the GPU path is covered by -m gpu); what is
under test is the partition and the reduction."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from conftest import ROOT, PKG


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _trial_nmse(sbce, trial, varn):
    from oracle.em_reduced import em_reduced, nmse
    b = sbce.signal_model.synthetic_batch(1, 2, 2, 4, 8, 12, 4, varn, seed=1000 + trial)
    aps = sbce.qam.all_possible_symbols(b["cons"], 2)
    th = em_reduced(b["y_d"][0], b["y_p"][0], b["u_p"][0], b["psi_d"][0].T, aps, varn, 2,
                    b["theta0"][0])
    return nmse(th, b["h"][0])


def _worker(rank, world, port, n_trials, varns, out):
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sbce = importlib.import_module(PKG)
    acc = sbce.distributed.Accumulators(len(varns))
    for pt, varn in enumerate(varns):
        mine = sbce.distributed.shard(n_trials, world, rank)
        acc.add(pt, [_trial_nmse(sbce, int(i), varn) for i in mine])
    acc.allreduce(dist)
    out[rank] = acc.pack().tolist()
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 4])
def test_sharded_sweep_matches_single_process(sbce, world):
    n_trials, varns = 7, [1.0, 0.1]
    ref = sbce.distributed.Accumulators(len(varns))
    for pt, varn in enumerate(varns):
        ref.add(pt, [_trial_nmse(sbce, i, varn) for i in range(n_trials)])
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_worker, args=(world, _free_port(), n_trials, varns, out), nprocs=world, join=True)
    for r in range(world):
        got = sbce.distributed.Accumulators(len(varns)).unpack(np.array(out[r]))
        assert np.array_equal(got.count, ref.count)
        assert np.allclose(got.mean_nmse(), ref.mean_nmse(), rtol=1e-14, atol=0)


def _oracle_em_batch(calls):
    """sweeps.em_batch stand-in: the oracle twin of each SNR-script EM per trial (per-trial or
    scalar varn), recording (mode, trials) of every call."""
    from test_oracle import _oracle_snr_em

    def fake(y_d, y_p, psi_d, u_p, cons, varn, itera, theta0, mode="soft", partition_r=0,
             h_true=None, **kw):
        calls.append((mode, len(y_d)))
        vt = np.broadcast_to(np.asarray(varn, dtype=float), (len(y_d),))
        th = np.stack([_oracle_snr_em(mode, y_d[b], y_p[b], psi_d[b].T, u_p[b], cons, vt[b], itera,
                                      theta0[b], None if h_true is None else h_true[b],
                                      partition_r) for b in range(len(y_d))])
        return dict(theta=th, status=np.zeros(len(y_d), dtype=np.int32))
    return fake


def _snr_sweep_worker(rank, world, port, monte_iter, out):
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    dist.init_process_group("gloo", rank=rank, world_size=world)
    sbce = importlib.import_module(PKG)
    calls, reduces = [], []
    sbce.sweeps.em_batch = _oracle_em_batch(calls)
    real = dist.all_reduce

    def counted(t, *a, **kw):
        reduces.append(t.numel())
        return real(t, *a, **kw)
    dist.all_reduce = counted
    snr, curves = sbce.sweeps.nmse_vs_snr(monte_iter=monte_iter, seed=0)
    dist.all_reduce = real
    out[rank] = dict(curves={k: v.tolist() for k, v in curves.items()}, calls=calls,
                     reduces=reduces)
    dist.barrier()
    dist.destroy_process_group()


def test_snr_sweep_driver_world2_matches_world1(sbce, monkeypatch):
    """sweeps.nmse_vs_snr (the north-star NMSE-vs-SNR figure, SNR/all_Detectors.py:362-395) under
    a real gloo world of 2: each rank runs its shard of the replayed trials (ONE call per detector
    with the SNR axis batched), ONE all-reduce carries every (detector, SNR) accumulator, and the
    five curves equal the world-1 run at 1e-14.  The oracle stands in for the device."""
    monte_iter = 3
    calls1 = []
    monkeypatch.setattr(sbce.sweeps, "em_batch", _oracle_em_batch(calls1))
    _, ref = sbce.sweeps.nmse_vs_snr(monte_iter=monte_iter, seed=0)
    assert [c[1] for c in calls1] == [monte_iter * 6] * 5          # 5 calls: every SNR point
    mgr = mp.Manager()
    out = mgr.dict()
    mp.spawn(_snr_sweep_worker, args=(2, _free_port(), monte_iter, out), nprocs=2, join=True)
    trials = 0
    for r in range(2):
        got = out[r]
        assert len(got["reduces"]) == 1 and got["reduces"][0] == 5 * 6 * 3   # nmse, count, flags
        trials += got["calls"][0][1]
        for mode, curve in ref.items():
            assert np.allclose(got["curves"][mode], curve, rtol=1e-14, atol=0), (r, mode)
    assert trials == monte_iter * 6


def test_shard_partition_is_exact(sbce):
    for n in (1, 7, 1000):
        for world in (1, 2, 3, 8):
            parts = [sbce.distributed.shard(n, world, r) for r in range(world)]
            allidx = np.sort(np.concatenate(parts))
            assert np.array_equal(allidx, np.arange(n))
    with pytest.raises(ValueError):
        sbce.distributed.shard(10, 2, 2)


class _StubDist:
    """Initialised process group stand-in: records the device of the all-reduce buffer."""

    class ReduceOp:
        SUM = "sum"

    def __init__(self, backend):
        self.backend, self.devices = backend, []

    def is_available(self):
        return True

    def is_initialized(self):
        return True

    def get_backend(self):
        return self.backend

    def all_reduce(self, t, op=None):
        self.devices.append(t.device)


def test_collective_device_follows_backend(sbce, monkeypatch):
    """RCCL ("nccl") reduces device tensors only: with that backend the accumulator vector
    must go to the current HIP device; gloo keeps it on the host."""
    import torch
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 3)
    assert sbce.distributed.collective_device(_StubDist("nccl")) == torch.device("cuda", 3)
    assert sbce.distributed.collective_device(_StubDist("gloo")) is None


def test_allreduce_uses_collective_device_by_default(sbce, monkeypatch):
    import torch
    seen = []

    def fake(dist):
        seen.append(dist.get_backend())
        return torch.device("cpu")        # stands in for the HIP device on a CPU-only host
    monkeypatch.setattr(sbce.distributed, "collective_device", fake)
    acc = sbce.distributed.Accumulators(2, n_iters=1)
    acc.add(0, [0.5, 0.25], llf_values=[[1.0], [2.0]])
    stub = _StubDist("nccl")
    acc.allreduce(stub)                   # what every sweep does: no explicit device
    assert seen == ["nccl"] and stub.devices == [torch.device("cpu")]
    assert acc.count.tolist() == [2.0, 0.0]
    # an explicit device wins and skips the backend query
    acc.allreduce(_StubDist("nccl"), device="cpu")
    assert seen == ["nccl"]


# ---------------------------------------------------------------- bench.py --gpus N launcher
def _bench():
    import importlib
    import sys
    if ROOT not in sys.path:
        sys.path.insert(0, ROOT)
    return importlib.import_module("bench")


def test_bench_rank_envs():
    """bench.launch_ranks gives rank r of N torchrun's variables: RANK = LOCAL_RANK = r (GPU r),
    WORLD_SIZE = N, rendezvous on 127.0.0.1."""
    b = _bench()
    envs = b.rank_envs(4, 29555, base={"PATH": "/usr/bin", "HSA_ENABLE_IPC_MODE_LEGACY": "0"})
    assert [e["RANK"] for e in envs] == ["0", "1", "2", "3"]
    assert [e["LOCAL_RANK"] for e in envs] == ["0", "1", "2", "3"]
    for e in envs:
        assert e["WORLD_SIZE"] == "4" and e["LOCAL_WORLD_SIZE"] == "4"
        assert e["MASTER_ADDR"] == "127.0.0.1" and e["MASTER_PORT"] == "29555"
        assert e["PATH"] == "/usr/bin" and e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"


def test_bench_gpus_must_match_world_size():
    b = _bench()
    assert b.check_world(b.parse_args(["--gpus", "4"]), env={"WORLD_SIZE": "4"}) == 4
    assert b.check_world(b.parse_args([]), env={"WORLD_SIZE": "2"}) == 2
    assert b.check_world(b.parse_args([]), env={}) == 1
    with pytest.raises(SystemExit) as e:
        b.check_world(b.parse_args(["--gpus", "8"]), env={"WORLD_SIZE": "1"})
    assert e.value.code == 2


def _run_bench(args, env_extra=None):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], env=env,
                       capture_output=True, text=True, timeout=300)
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return r, lines


@pytest.mark.parametrize("n", [2, 3])
def test_bench_gpus_n_launches_n_ranks(n):
    """`bench.py --gpus N` with no launcher starts N ranks (gloo self-test: the launcher, the
    host barriers, the max-over-ranks clock and the accumulator all-reduce) and prints ONE line
    with n_gpus = N whose accumulators cover every rank."""
    r, lines = _run_bench(["--gpus", str(n), "--selftest", "--steps", "2", "--warmup", "1"])
    assert r.returncode == 0, r.stderr[-2000:]
    assert len(lines) == 1
    line = lines[0]
    assert line["n_gpus"] == n and line["steps"] == 2 and line["scaling"] == "weak"
    assert line["trials_total"] == 8 * n
    assert line["nmse_mean"] == pytest.approx(0.5 * sum(range(1, n + 1)) / n)


def test_bench_mismatched_launch_fails():
    """Under a launcher (WORLD_SIZE set) a disagreeing --gpus exits non-zero before any work."""
    r, lines = _run_bench(["--gpus", "4", "--selftest"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert r.returncode == 2 and not lines
    assert "WORLD_SIZE=2" in r.stderr


def test_bench_reference_structured_work_model_follows_estep():
    """The reference-structured CPU baseline extrapolates by T_d J K^2 with J = the hypotheses the
    workload's E-step visits: M^n_tx (exact / log-max), the PM list M^(p+1) (PMd/PM.py:74-92)."""
    b = _bench()
    assert b.hypotheses_per_symbol("soft", 4, 16) == 16 ** 4
    assert b.hypotheses_per_symbol("hard", 2, 4) == 16
    assert b.hypotheses_per_symbol("pm_soft", 8, 16, 1) == 16        # cfg2: p = int(1/4) = 0
    assert b.hypotheses_per_symbol("pm", 4, 4, 2) == 16              # p = int(2/2) = 1
    assert b.host_threads() >= 1


def test_bench_panel_factor_work_model():
    """bench.panel_factor_mfma_per_trial counts the FP64 MFMAs the wide schedule's factor launches
    issue (csrc/chol.hip): cfg1's L = 260 gives 5216 per trial; one 32-column panel of 2 tiles
    has TRSM A + B-part update of tile 1 only (32), no TRSM B and no pre-update."""
    b = _bench()
    assert b.panel_factor_mfma_per_trial(260) == 5216
    assert b.panel_factor_mfma_per_trial(32) == 32
    # L = 48: panel 0 has 3 tiles (TRSM A + update of tiles 1, 2: 64; TRSM B of tile 2: 20);
    # panel 1 (odd, one tile) only its rank-32 pre-update of tile 0's lower half (24)
    assert b.panel_factor_mfma_per_trial(48) == 64 + 20 + 24
