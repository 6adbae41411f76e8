#!/usr/bin/env python3
"""Headline benchmark: vectorised microRTS env-steps/s on MI355X (BASELINE.json metric).

Workload (BASELINE.json configs[2]): maps/16x16/basesWorkers16x16.xml, 4096
self-play games per GPU (8192 player slots), UTT VERSION_ORIGINAL + CANCEL_BOTH, max_steps 2000,
masked uniform random policy (Philox, seed 0x5EEDC0DE), legal-action masks and observations written
every step.  One "step" = one batched gameStep of every game on every GPU: the step kernel (decode ->
issueSafe -> cycle -> WinLoss -> auto-reset -> observation -> masks) consumes the int32 action tensor
in HBM; the synthetic random-policy actions of the next step are sampled from the masks it writes and
written back to that tensor by the same launch (--policy fused, the default: mrts_step_fused_dev,
bit-identical to the standalone policy kernel) or by a separate policy launch before each step
(--policy kernel: what an external agent's launch would look like).  The JSON line also carries the
other form's throughput over the next K steps ("other_policy_form").  Default mask mode "delta":
the mask / action tensors are persistent and only rows that changed are rewritten (identical
contents to a full rewrite, tested); --mask-mode full rewrites every byte.  An env-step is one game-cycle
(a self-play game counts once, not twice).  Inputs are resident in HBM; nothing crosses PCIe in
the timed region.

Multi-GPU: one process per GPU (torch.distributed.run), each rank steps its own disjoint shard of
games (weak scaling, no collective in the step); barrier + synchronize bracket the timed region and
the max time over ranks is reported.  --gather-obs [allgather|learner] adds the north-star RCCL
exchange of the observation tensor every step (int16 transport, double-buffered, on its own stream so
it overlaps the next step; all-gather to every rank or gather to rank 0) — not the default, since
nothing in the step consumes it.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "env-steps/s (random policy) at N envs/GPU, 1/2/4/8 MI355X; bit-exact vs Java"
MAP = "maps/16x16/basesWorkers16x16.xml"
SEED = 0x5EEDC0DE
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md: 8.0 TB/s)


# BASELINE.json configs: (map, self-play games per GPU, partial observability, max_units)
# c5: the 32x32 map's live units never exceeded 32 in 2500-step random-policy games (oracle); a
# 256-unit bound (error flags checked after the run) lets all 2048 games be resident at once.
CONFIGS = {
    "c2": ("maps/8x8/basesWorkers8x8.xml", 1024, False, 0),
    "c3": (MAP, 4096, False, 0),
    "c5": ("maps/BWDistantResources32x32.xml", 2048, True, 256),
    "c5-exact": ("maps/BWDistantResources32x32.xml", 2048, True, 0),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--burnin", type=int, default=1000,
                    help="untimed steps from reset before warmup: the timed window sees mid-episode unit counts")
    ap.add_argument("--config", choices=sorted(CONFIGS) + ["c1"], default="c3",
                    help="BASELINE.json workload preset (c3 = the headline; c2 / c5 = the other single-GPU configs; "
                         "c1 = one bot-vs-bot env, RandomBiasedAI x 2, with the CPU oracle beside it)")
    ap.add_argument("--envs", type=int, default=None, help="self-play games per GPU (default: the preset's)")
    ap.add_argument("--map", default=None)
    ap.add_argument("--mask-mode", choices=["delta", "full"], default="delta",
                    help="delta: the persistent mask tensor is updated in place (only changed rows written); "
                         "full: every mask byte is rewritten each step")
    ap.add_argument("--gather-obs", nargs="?", const="allgather", choices=["allgather", "learner"], default=None,
                    help="per-step RCCL exchange of the observation tensor (int16 transport, on its own stream, "
                         "overlapped with the next step): all-gather to every rank, or gather to rank 0")
    ap.add_argument("--policy", choices=["kernel", "fused", "uniform", "uniform-split"], default=None,
                    help="kernel: the masked random policy is its own launch before each step; fused: the step "
                         "kernel samples the next step's actions from the masks it writes (mrts_step_fused_dev, "
                         "same Philox stream, bit-identical actions); uniform: SURVEY.md §8(d)'s c2 workload, "
                         "unmasked uniform rows for every cell and no masks, drawn and written by the step kernel "
                         "itself (mrts_step_uniform_dev); uniform-split: the same rows from their own kernel launch "
                         "before each step (mrts_policy_uniform_dev).  Default: uniform for c2, fused otherwise")
    ap.add_argument("--launch", choices=["native", "graph", "eager"], default=None,
                    help="how the K timed steps are enqueued: native = one mrts_rollout_fused_dev call (K launches "
                         "from C++; fused policy only, the default there), graph = replay of a captured hipGraph "
                         "(the default for --policy kernel), eager = one Python call per step")
    ap.add_argument("--no-graph", action="store_true", help="alias of --launch eager")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-gather-window", action="store_true",
                    help="skip the second timed window with the per-step RCCL observation all-gather (with_gather)")
    ap.add_argument("--no-exchange-u8", dest="exchange_u8", action="store_false",
                    help="exchange the observation as int16 even where every value fits a byte")
    ap.add_argument("--gather-timeout", type=float, default=180.0,
                    help="seconds the with_gather window may take on a rank before every rank gives it up: rank 0 "
                         "prints the line with with_gather = {error} and all ranks exit 0 (a hung collective must "
                         "not cost the headline line)")
    ap.add_argument("--no-compare", action="store_true", help="skip the other policy form's comparison window")
    ap.add_argument("--utt", type=int, choices=[1, 2], default=1,
                    help="UnitTypeTable version: 1 VERSION_ORIGINAL (the traces', SURVEY.md §8(d)), 2 VERSION_ORIGINAL_"
                         "FINETUNED (SURVEY.md §8(d)'s secondary sweep); CANCEL_BOTH either way")
    ap.add_argument("--no-full-contract", action="store_true",
                    help="skip the full_contract window (full mask rewrite + separate policy launch, one launch per step)")
    ap.add_argument("--gather-window", choices=["records", "tensor"], default="records",
                    help="with_gather: records = all-gather of the compact game records (default); tensor = the "
                         "per-step all-gather of the uint8 / int16 observation tensor")
    ap.add_argument("--records-steps", type=int, default=0,
                    help="steps per launch of the records window (0 = the K steps in one launch)")
    ap.add_argument("--cpu-threads", type=int, default=None,
                    help="threads of the all-cores CPU baseline (default: every CPU this process may use, capped by "
                         "the cgroup's CPU quota)")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="c3 at N = 1: skip the c2 and c5 sub-blocks (each BASELINE single-GPU config run as a child "
                         "bench.py with the same K / W, its line nested under configs)")
    ap.add_argument("--pmc-traffic", type=float, default=None,
                    help="HBM bytes per step-kernel launch from a rocprofv3 --pmc pass (profiles/), for roofline.traffic")
    a = ap.parse_args()
    if a.config == "c1":
        a.map = a.map or "maps/4x4/base4x4.xml"
        return a
    m, e, po, mu = CONFIGS[a.config]
    a.map = a.map or m
    a.envs = a.envs or e
    a.po = po
    a.max_units = mu
    if a.policy is None:
        a.policy = "uniform" if a.config == "c2" else "fused"
    if a.no_graph:
        a.launch = "eager"
    if a.launch is None:
        a.launch = "native" if a.policy in ("fused", "uniform", "uniform-split") else "graph"
    if a.launch == "native" and a.policy not in ("fused", "uniform", "uniform-split"):
        ap.error("--launch native needs --policy fused or uniform")
    if a.launch == "graph" and a.gather_obs:
        # a torch.cuda.graph capture of torch.distributed collectives (why it aborted)
        ap.error("--launch graph cannot capture the --gather-obs collectives; use --launch eager")
    return a


class _FenceFreeEvent:
    """A HIP timing event created with hipEventDisableSystemFence: recording it does not add a
    system-scope release fence (cache write-back) in front of the bracketed kernel, so an event pair
    around one launch measures that kernel plus only its dispatch.  Bound with ctypes to the HIP
    runtime torch already loaded (one runtime per process); torch.cuda.Event is the fallback."""

    _hip = None

    @classmethod
    def runtime(cls):
        if cls._hip is None:
            import ctypes

            path = None
            with open("/proc/self/maps") as f:
                for line in f:
                    if "libamdhip64.so" in line:
                        path = line.split()[-1]
                        break
            if path is None:
                raise OSError("libamdhip64 not loaded")
            hip = ctypes.CDLL(path)
            hip.hipEventCreateWithFlags.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_uint]
            hip.hipEventRecord.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
            hip.hipEventElapsedTime.argtypes = [ctypes.POINTER(ctypes.c_float), ctypes.c_void_p, ctypes.c_void_p]
            hip.hipEventDestroy.argtypes = [ctypes.c_void_p]
            cls._hip = hip
        return cls._hip

    def __init__(self):
        import ctypes

        self.ctypes = ctypes
        self.h = ctypes.c_void_p()
        if self.runtime().hipEventCreateWithFlags(ctypes.byref(self.h), 0x20000000) != 0:  # hipEventDisableSystemFence
            raise OSError("hipEventCreateWithFlags failed")

    def record(self, stream):
        if self._hip.hipEventRecord(self.h, self.ctypes.c_void_p(stream.cuda_stream)) != 0:
            raise OSError("hipEventRecord failed")

    def elapsed_time(self, end):
        ms = self.ctypes.c_float()
        if self._hip.hipEventElapsedTime(self.ctypes.byref(ms), self.h, end.h) != 0:
            raise OSError("hipEventElapsedTime failed")
        return ms.value


def code_sha256():
    """SHA-256 of the gfx950 code object of the libmrts.so this process runs: the counter files name the
    kernels' machine code they describe (microrts_amd._lib.device_code_sha256)."""
    from microrts_amd import _lib

    return _lib.device_code_sha256()


def cgroup_cpus():
    """CPUs' worth of time the cgroup grants this process (cpu.max quota / period), or None."""
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            q, per = open(path).read().split()[:2]
            if q != "max":
                return float(q) / float(per)
        except (OSError, ValueError):
            pass
    try:
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        if q > 0:
            return q / per
    except (OSError, ValueError):
        pass
    return None


def all_cores():
    """SURVEY.md §8(d)'s "all cores": the CPUs this process may run on (affinity), capped by the
    cgroup's CPU quota when one is set (more threads than that only time-share the same cores)."""
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count() or 1
    q = cgroup_cpus()
    return max(1, min(usable, int(q))) if q else usable


def host_info():
    """The host the CPU baseline ran on: logical CPUs (nproc), the CPUs this process may use, the
    cgroup's CPU quota, the model."""
    model = None
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = os.cpu_count()
    return {"nproc": os.cpu_count(), "usable_cpus": usable, "cgroup_cpu_quota": cgroup_cpus(), "cpu_model": model}


def cpu_baseline(map_path, threads, burnin, uniform=False, po=False, runs=5, utt=1):
    """The CPU oracle (C++ restatement of the Java engine; the JVM is not available) running the
    same workload: VecClient self-play + getMasks + the same Philox policy (or c2's uniform rows),
    partially observable views for c5, std::thread shards over games — on all cores (`threads`,
    all_cores()) and on one thread, the sequential loop of JNIGridnetVecClient.gameStep
    (SURVEY.md §8(d)).  Median of `runs` runs; a bounded sample (a few seconds per run)."""
    import statistics

    from tests import oracle_py

    L = oracle_py.load()
    games_per_thread, steps = 48, (100 if po else 300)
    games = games_per_thread * threads
    flags = (1 if uniform else 0) | (2 if po else 0) | (utt << 2)
    rates = [games * steps / L.oref_bench3(map_path.encode(), games, steps, threads, SEED, burnin, flags) for _ in range(runs)]
    ones = [games_per_thread * steps / L.oref_bench3(map_path.encode(), games_per_thread, steps, 1, SEED, burnin, flags)
            for _ in range(3)]
    what = ("uniform rows, no masks" if uniform else "masks + masked policy" + (", partially observable views" if po else "")) + \
        (f", UTT version {utt}" if utt != 1 else "")
    return {
        "value": statistics.median(rates),
        "unit": "env-steps/s",
        "cores": threads,
        "kind": "port",
        "sample": f"{games} self-play games x {steps} timed steps after {burnin} untimed, {threads} threads (same map, "
                  f"{what}); median of {runs} runs {[round(r) for r in rates]}; 1 thread: "
                  f"{statistics.median(ones):.0f} env-steps/s (median of 3)",
        "runs": rates,
        "one_thread": statistics.median(ones),
        "host": host_info(),
    }


def cpu_baseline_c1(map_path, runs=5, steps=200_000, burnin=1000):
    """BASELINE config c1: one JNIBotClient env, RandomBiasedAI vs RandomBiasedAI (seeded
    java.util.Random 42), bot-only VecClient auto-reset; env-steps/s, 1 thread, median of `runs`."""
    import statistics

    from tests import oracle_py

    L = oracle_py.load()
    rates = [steps / L.oref_bench_bots(map_path.encode(), steps, 42, burnin) for _ in range(runs)]
    return {"value": statistics.median(rates), "unit": "env-steps/s", "cores": 1, "kind": "port",
            "sample": f"1 env x {steps} timed gameSteps after {burnin} untimed (JNIBotClient semantics, RandomBiasedAI x 2, "
                      f"java.util.Random seed 42); median of {runs} runs {[round(r) for r in rates]}",
            "runs": rates, "host": host_info()}


def run_with_deadline(fn, seconds, on_timeout):
    """fn() with a watchdog: if it has not returned after `seconds`, on_timeout() runs on the watchdog
    thread (bench.py's: print the line without the window, exit every rank).  The timer is cancelled
    when fn returns or raises."""
    import threading

    watchdog = threading.Timer(seconds, on_timeout)
    watchdog.daemon = True
    watchdog.start()
    try:
        return fn()
    finally:
        watchdog.cancel()


def gather_window(env, a, xg, one_step, base, total_games, world, mdist, torch, dist, mode=None):
    """K steps with the observation all-gather after every step, one step launch per step (a per-step
    consumer cannot use multi-step launches); the barrier + synchronize bracket and max over ranks of
    the headline window.  -> the JSON block.  Full observability over RCCL: the native form
    (mdist.NativeExchange: the K steps and their all-gathers enqueued by libmrts, the step kernel
    writing the int16 transport, the collectives on the handle's own stream).  Otherwise (partially
    observable views, gloo) one_step with xg["buf"] (Python enqueues each step and its collective).
    No hipGraph capture: a capture that fails leaves RCCL work events recorded in a capturing stream,
    and the process group's watchdog thread then aborts the whole process."""
    native_ok = (mode is not None and dist.get_backend() != "gloo" and not a.po and a.launch == "native"
                 and (mode["fused"] or mode["uni_fused"]))
    nx = None
    if native_ok:
        try:
            # uint8 transport where every observation value fits a byte (c3's 16x16 maps), else int16
            nx = mdist.NativeExchange(env, u8="auto" if a.exchange_u8 else False)
        except Exception as ex:  # e.g. no RCCL library to bind: every rank must take the same path
            print(f"bench: native exchange unavailable ({ex!r}); torch collectives", file=sys.stderr)
        flag = torch.tensor([1 if nx is not None else 0], device=env.device)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        native_ok = bool(flag.item())
    u8 = bool(native_ok and nx.u8)
    if native_ok:

        def run(first, n):
            if mode["fused"]:
                nx.rollout_fused(SEED, first + 1, n)
            else:
                nx.rollout_uniform(SEED, first, n)

        run(base, 3)  # untimed: the first collectives set up the communicator's channels
        # the K steps and their collectives as one graph (RCCL's host cost per call would pace the
        # steps otherwise: ~30 us of host work per step against a 9-22 us step)
        nx.capture(lambda: run(base + 3, a.steps))
        torch.cuda.synchronize(env.device)
        nx.replay()  # warm replay (the first replay carries one-off costs)
        torch.cuda.synchronize(env.device)
        if world > 1:  # (one rank: nothing to wait for; the headline window does the same)
            dist.barrier()
        torch.cuda.synchronize(env.device)
        t0 = time.perf_counter()
        nx.replay()
        torch.cuda.synchronize(env.device)
        if world > 1:  # (one rank: nothing to wait for; the headline window does the same)
            dist.barrier()
        t = mdist.max_over_ranks(time.perf_counter() - t0, env.device)
        how = ("native: mrts_rollout_*_exchange_dev enqueues each step launch and its ncclAllGather on the handle's own "
               "RCCL communicator, captured once as a graph by libmrts (mrts_capture_begin / _end) and replayed")
    else:
        gb = mdist.ObservationGather(env.obs.shape, env.device, mode="allgather")
        xg["buf"] = gb
        try:
            for k in range(3):  # untimed: the first collectives set up the communicator's channels
                one_step(base + k)
            gb.wait()
            torch.cuda.synchronize(env.device)
            if world > 1:  # (one rank: nothing to wait for; the headline window does the same)
                dist.barrier()
            torch.cuda.synchronize(env.device)
            t0 = time.perf_counter()
            for k in range(a.steps):
                one_step(base + 3 + k)
            gb.wait()  # the last step's exchange belongs to the window
            torch.cuda.synchronize(env.device)
            if world > 1:  # (one rank: nothing to wait for; the headline window does the same)
                dist.barrier()
            t = mdist.max_over_ranks(time.perf_counter() - t0, env.device)
        finally:
            xg["buf"] = None
            env.set_obs16(None)
        how = "eager: Python enqueues each step and its collective (torch.distributed)"
    return {
        "value": total_games * a.steps / t,
        "ms_per_step": 1e3 * t / a.steps,
        "collective": f"all-gather of the {'uint8' if u8 else 'int16'} observation tensor every step (RCCL, ring over "
                      "xGMI), comm stream overlapping the next step; " +
                      ("uint8 written by the step kernel (every value < 256, checked at create)" if u8 else
                       "int16 written by the step kernel" if not a.po else "narrowing copy (partially observable planes)"),
        "payload_bytes_per_rank": env.obs.numel() * (1 if u8 else 2),  # one rank's observation, per step
        "launch": "one step launch per step (a per-step consumer cannot use multi-step launches); " + how,
    }


def records_window(env, a, mode, base, total_games, world, mdist, torch, dist):
    """SURVEY.md §8e's second curve with the compact observation exchange: the same K
    steps (multi-step launches of a.records_steps steps each, 0 = one launch), and after each launch an
    in-place RCCL all-gather of every step's game records (the unit lists GameState.getVectorObservation
    reads) on the handle's own stream, overlapping the next launch; barrier + synchronize bracket and
    max over ranks as the headline.  The receiver's render of every rank's observations (uint8) is
    timed separately per step (render_ms_per_step)."""
    rx = mdist.RecordExchange(env, units_per_record=64, steps_per_launch=a.records_steps)
    # every step's reward / done too (mrts_set_step_responses): with the records, each step's full Responses
    env.set_step_responses(max(3, a.steps))

    def run(first, n):
        if mode["fused"]:
            return rx.rollout_fused(SEED, first + 1, n)
        return rx.rollout_uniform(SEED, first, n)

    run(base, 3)  # untimed: the first collectives set up the communicator's channels
    rx.buffer(a.steps)
    torch.cuda.synchronize(env.device)
    if world > 1:  # (one rank: nothing to wait for; the headline window does the same)
        dist.barrier()
    torch.cuda.synchronize(env.device)
    t0 = time.perf_counter()
    off = run(base + 3, a.steps)
    torch.cuda.synchronize(env.device)
    if world > 1:  # (one rank: nothing to wait for; the headline window does the same)
        dist.barrier()
    t = mdist.max_over_ranks(time.perf_counter() - t0, env.device)
    # the receiving side: every rank's observations of one step back as uint8 planes
    S = env.dims[0]
    b8 = torch.int8 if a.po else torch.uint8  # partially observable: a dead unit in a view can show hp <= 0
    out8 = torch.zeros((world * S,) + tuple(env.obs.shape[1:]), dtype=b8, device=env.device)
    n_r = min(5, a.steps)
    e0, e1 = _FenceFreeEvent(), _FenceFreeEvent()
    cur = torch.cuda.current_stream(env.device)
    rx.render(off, 0, out8)
    e0.record(cur)
    for j in range(n_r):
        rx.render(off, j, out8)
    e1.record(cur)
    torch.cuda.synchronize(env.device)
    render_ms = e0.elapsed_time(e1) / n_r
    # the render of an 8-rank step on this one GPU — what each rank of c4 writes per step if it materialises every
    # rank's observations — over an 8-rank receive buffer laid out as one chunk of an 8-rank all-gather
    # ([rank][step][game][words], rank stride K x games x words): rank r's place holds this rank's records of each
    # step with the games rotated by r (a rank stride of 0 would read one rank's records 8 times, cache-hot)
    K = a.steps
    G2, per = S // 2, (S // 2) * rx.words
    own = torch.stack([rx.recv[int(off[j][0]):int(off[j][0]) + per] for j in range(K)]).view(K, G2, rx.words)
    rx8 = torch.empty((8, K, G2, rx.words), dtype=torch.int32, device=env.device)
    for r in range(8):
        rx8[r] = torch.roll(own, -r, 1)
    rx8 = rx8.view(-1)
    del own
    out8r = torch.zeros((8 * S,) + tuple(env.obs.shape[1:]), dtype=b8, device=env.device)
    env.render_records(rx8, 0, K * per, 8, out8r)
    e0.record(cur)
    for j in range(n_r):
        env.render_records(rx8, j * per, K * per, 8, out8r)
    e1.record(cur)
    torch.cuda.synchronize(env.device)
    render8_ms = e0.elapsed_time(e1) / n_r
    del out8r
    # a learner's batch in MicroRTS-Py's one-hot layout straight from the records: B random
    # slots of the 8-rank volume per step, from the same 8-rank buffer
    onehot = {}
    if not a.po:
        gsel = torch.Generator(device="cpu").manual_seed(1)
        for B in (1024, 2048, S):  # per step; one launch for the window's K steps
            sel = torch.randint(0, 8 * S, (K * B,), generator=gsel).to(torch.int32).to(env.device)
            so = torch.tensor([[j * per, K * per] for j in range(K) for _ in range(B)], dtype=torch.int64, device=env.device)
            oh = env.render_records_onehot(rx8, 0, 0, sel, step_off=so)
            e0.record(cur)
            env.render_records_onehot(rx8, 0, 0, sel, oh, step_off=so)
            e1.record(cur)
            torch.cuda.synchronize(env.device)
            us = 1e3 * e0.elapsed_time(e1) / K
            onehot[str(B)] = {"us_per_step": us, "bytes_per_step": oh.numel() / K, "GBps": oh.numel() / K / (us * 1e-6) / 1e9}
            del oh
    del rx8
    env.set_step_responses(0)
    rec_bytes = (S // 2) * rx.words * 4
    return {
        "value": total_games * a.steps / t,
        "ms_per_step": 1e3 * t / a.steps,
        "collective": "in-place RCCL all-gather (ring over xGMI) of each launch's compact game records: per game and step "
                      + (f"{rx.words} words = the units of either view (<= 64) x 2 words (cell, hp, resources, type, owner, "
                         "snapshot membership and seen action per view), the inputs of "
                         "PartiallyObservableGameState.getVectorObservation" if a.po else
                         f"{rx.words} words = live units (<= 64) x (cell, hp, resources, type, owner, action), the inputs of "
                         "GameState.getVectorObservation") + "; on the handle's own stream, overlapping the next launch",
        "payload_bytes_per_rank_per_step": rec_bytes,
        "observation_bytes_per_rank_per_step": {"uint8": env.obs.numel(), "int32": 4 * env.obs.numel()},
        "render_ms_per_step": render_ms,
        "render_ms_per_step_8_ranks": render8_ms,
        "render_8_ranks_buffer": "one chunk of an 8-rank all-gather: rank r's place = this rank's records rotated by r games, "
                                 "rank stride K x games x words (not a stride-0 re-read of one rank)",
        "render_GBps_8_ranks": 8 * env.obs.numel() / (render8_ms * 1e-3) / 1e9,
        "onehot_batch": onehot or None,
        "onehot_batch_note": "mrts_render_records_onehot_dev: B random slots of the 8-rank volume at each of the window's K "
                             "steps (an 8-rank receive buffer: rank r's place = this rank's records rotated by r games, real "
                             "rank stride), as MicroRTS-Py one-hot uint8 [K x B][H][W][F] (a learner's minibatch), ONE launch, "
                             "timed alone (per step = / K); it does not overlap the step launches, whose waves hold every "
                             "SIMD's VGPRs (4 x 128) and the CUs' LDS (16 x 10 KB): tools/consumer_overlap.py",
        "render": f"mrts_render_records_dev: all {world} ranks' observations of one step rebuilt as {'int8' if a.po else 'uint8'} "
                  f"[{world * S}, {env.dims[3]}, {env.dims[1]}, {env.dims[2]}] (not in value: a consumer may read the "
                  "records directly)",
        "responses": "every step's reward / done written to a per-step ring inside the launches (mrts_set_step_responses; "
                     "rank-local), so with the records each step's full Responses (JNIGridnetVecClient.gameStep) is available",
        "steps_per_launch": a.records_steps or "all",
        "launch": "multi-step launches (each game's state in LDS), every step's records written by the step kernel",
    }


def full_contract_window(a, sh, local, base, total_games, world, mdist, torch, dist, DeviceVecEnv):
    """VERDICT r3 #3a / r4 #6 — SURVEY.md §8(d)'s byte contract, as the Java client moves it: every mask
    byte rewritten each step (JNIGridnetClientSelfPlay.java:196-209, mask_delta off), the policy as its own
    launch reading the full masks and writing every action row, one step launch per step (a per-step
    consumer), on a second handle with the headline's shard.  §8(d) excludes policy generation and reports
    it separately: the step kernel and the policy kernel are timed apart (fence-free events around each
    launch of an eager pass), so the §8(d) fraction is given over the step kernel's time (step_only) and
    over the whole step + policy window (step_plus_policy).  A fused variant (the step kernel samples the
    next rows itself, masks still fully rewritten, one launch per step) shows what full masks alone cost.
    -> the JSON block."""
    import numpy as np

    from microrts_amd import UnitTypeTable

    env = DeviceVecEnv(sh["n_slots"], 0, 2000, [os.path.join(ROOT, a.map)] * sh["n_slots"], device=local, seed=SEED,
                       partial_obs=a.po, max_units=a.max_units, slot_id_base=sh["slot_id_base"], mask_delta=False,
                       source_bits=False, utt=UnitTypeTable(a.utt, 1))
    S, H, W, C, K = env.dims
    env.reset()
    for k in range(a.burnin):
        env.random_policy(SEED, k)
        env.step()
    t_step = a.burnin
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(env.device)
    cap.wait_stream(torch.cuda.current_stream(env.device))
    with torch.cuda.graph(graph, stream=cap):  # kernels only: no collective in this graph
        for k in range(a.steps):
            env.random_policy(SEED, t_step + k)
            env.step()
    torch.cuda.synchronize(env.device)
    graph.replay()  # warm
    torch.cuda.synchronize(env.device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(env.device)
    t0 = time.perf_counter()
    graph.replay()
    torch.cuda.synchronize(env.device)
    if world > 1:
        dist.barrier()
    t = mdist.max_over_ranks(time.perf_counter() - t0, env.device)
    t_step += a.steps  # (the replays rerun the captured step indices; the policy stream does not care)
    # the two kernels apart: an eager pass with fence-free events around each launch
    cur = torch.cuda.current_stream(env.device)
    n_e = min(a.steps, 20)
    ev = [[_FenceFreeEvent() for _ in range(4)] for _ in range(n_e)]
    for k in range(n_e):
        ev[k][0].record(cur)
        env.random_policy(SEED, t_step + k)
        ev[k][1].record(cur)
        ev[k][2].record(cur)
        env.step()
        ev[k][3].record(cur)
    torch.cuda.synchronize(env.device)
    t_step += n_e
    pol_us = 1e3 * float(np.median([ev[k][0].elapsed_time(ev[k][1]) for k in range(n_e)]))
    stp_us = 1e3 * float(np.median([ev[k][2].elapsed_time(ev[k][3]) for k in range(n_e)]))
    # fused policy, full masks: one launch per step (not the steady delta state), timed like the headline
    env.random_policy(SEED, t_step)
    env.rollout_fused(SEED, t_step + 1, 2)  # warm
    t_step += 2
    torch.cuda.synchronize(env.device)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(env.device)
    t1 = time.perf_counter()
    env.rollout_fused(SEED, t_step + 1, a.steps)
    torch.cuda.synchronize(env.device)
    if world > 1:
        dist.barrier()
    tf = mdist.max_over_ranks(time.perf_counter() - t1, env.device)
    assert not env.error_flags().any()
    units = float(np.mean([env.dump_state(s)[4] for s in range(0, min(S, 64), 2)]))
    HW = H * W
    survey = S * (HW * 7 * 4 + C * HW * 4 + HW * K + (16 * units + 2 * HW + 16))
    env.close()
    step_s = t / a.steps
    # the bytes this leg moves through the L2's memory-side (fabric) request counters: the policy launch reads
    # every mask byte the step launch wrote, and the step re-reads every action row.  FETCH_SIZE / WRITE_SIZE
    # count Infinity-Cache (L3, 256 MiB) hits too (MI355X_MICROARCH.md, HBM section), so this is L2-fabric
    # traffic, an upper bound on HBM bytes — not HBM bytes (tools/profile_full_contract.sh +
    # tools/full_contract_pmc.py summarize)
    traffic = None
    pf = os.path.join(ROOT, "profiles", f"pmc_full_contract_{a.config}.json")
    if os.path.exists(pf) and a.utt == 1 and world == 1:
        pj = json.load(open(pf))
        if pj.get("gfx950_code_sha256") != code_sha256():
            traffic = {"note": f"{os.path.relpath(pf, ROOT)} was taken with other kernel code; not used"}
        elif pj.get("games") == sh["n_slots"] // 2:
            tb = pj["traffic_bytes_per_step"]
            traffic = {"l2_fabric_bytes_per_step": tb, "l2_fabric_GBps": tb / step_s / 1e9,
                       "what": "2 x FETCH_SIZE + WRITE_SIZE of the leg's policy + step launches: L2 memory-side requests, "
                               "Infinity-Cache hits included (the policy's re-read of the just-written masks fits the 256 MiB "
                               "L3), so an upper bound on HBM traffic, not a fraction of HBM peak",
                       "source": f"{os.path.relpath(pf, ROOT)} ({pj['tag']}: separate --pmc passes, same gfx950 code object)"}
    out = {
        "value": total_games * a.steps / t,
        "ms_per_step": 1e3 * step_s,
        "mask_mode": "full (every mask byte rewritten every step)",
        "policy": "separate masked-uniform policy launch per step (reads every mask byte, writes every action row)",
        "launch": "hipGraph replay of K x (policy launch + step launch)",
        "survey_8d_bytes_per_step": survey,
        "step_only": {"step_kernel_us": stp_us, "survey_8d_GBps": survey / (stp_us * 1e-6) / 1e9,
                      "survey_8d_frac": survey / (stp_us * 1e-6) / 1e9 / HBM_PEAK_GBS,
                      "timing": f"median of {n_e} step launches, fence-free HIP events around each (eager pass)"},
        "policy_kernel_us": pol_us,
        "step_plus_policy": {"survey_8d_GBps": survey / step_s / 1e9, "survey_8d_frac": survey / step_s / 1e9 / HBM_PEAK_GBS,
                             "timing": "wall clock of the graph replay (both kernels, launch gaps)"},
        "fused_full_masks": {"value": total_games * a.steps / tf, "ms_per_step": 1e3 * tf / a.steps,
                             "survey_8d_frac": survey / (tf / a.steps) / 1e9 / HBM_PEAK_GBS,
                             "launch": "mrts_rollout_fused_dev on the full-mask handle: one launch per step, the step kernel "
                                       "samples the next rows itself and rewrites every mask byte and every action row"},
        "note": "SURVEY.md §8(d): B = A + O + M + S per env-step (all action rows read, int32 observation, uint8 masks, "
                "live state); policy generation excluded from B and timed separately (policy_kernel_us)",
    }
    if traffic is not None:
        out["traffic"] = traffic
    return out


def child_env(environ):
    """The environment of a child bench.py run: a fresh one-rank run, so none of a launcher's rendezvous variables
    (under torch.distributed.run, TORCHELASTIC_USE_AGENT_STORE would make the child's process group wait as a
    client of a store that is not there)."""
    launcher = ("MASTER_ADDR", "MASTER_PORT", "RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "GROUP_RANK",
                "GROUP_WORLD_SIZE", "ROLE_RANK", "ROLE_NAME", "ROLE_WORLD_SIZE")
    return {k: v for k, v in environ.items() if k not in launcher and not k.startswith("TORCHELASTIC_")}


def other_configs(a, timeout=240.0):
    """the other single-GPU BASELINE configs in the driver's own line — c2 (configs[1]: 8x8, 1024
    games, unmasked uniform rows) and c5 (configs[4] per GPU: 32x32, 2048 partially observable games, masked
    policy) — each a child bench.py with the same K / W / burn-in, run after this process has released its
    handle and process group; its JSON line (value, ms_per_step, roofline with the matching-hash PMC file,
    cpu_baseline, ...) nested under its name.  When the driver's K is not 200, each of c2 / c3 / c5 also gets a
    quick K = 200 child without the CPU baseline (`configs.c2.k200`, `configs.c5.k200`, `configs.c3_k200`), the
    window the builder's own figures are quoted at.  A child that fails or overruns leaves {"error": ...} there."""
    import subprocess

    env = child_env(os.environ)

    def child(cfg, extra):
        cmd = [sys.executable, os.path.abspath(__file__), "--config", cfg, "--warmup", str(a.warmup), "--burnin", str(a.burnin)]
        cmd += extra
        t0 = time.perf_counter()
        try:
            p = subprocess.run(cmd, env=env, stdout=subprocess.PIPE, stderr=subprocess.PIPE, timeout=timeout, cwd=ROOT)
            lines = [ln for ln in p.stdout.decode().splitlines() if ln.startswith("{")]
            if p.returncode != 0 or not lines:
                r = {"error": f"exit {p.returncode}: {p.stderr.decode()[-400:]}"}
            else:
                r = json.loads(lines[-1])
        except subprocess.TimeoutExpired:
            r = {"error": f"timed out after {timeout:.0f} s"}
        r["command"] = " ".join(["python3", "bench.py"] + cmd[2:])
        r["run_s"] = time.perf_counter() - t0
        return r

    res = {}
    for cfg in ("c2", "c5"):
        res[cfg] = child(cfg, ["--steps", str(a.steps)])
    if a.steps != 200:
        # the bench default K = 200 beside the driver's K (round 5's c2 / c5 figures were K = 200 windows): the
        # timed window only (no CPU baseline, exchange, full-contract or comparison windows)
        quick = ["--steps", "200", "--no-cpu-baseline", "--no-gather-window", "--no-full-contract", "--no-compare",
                 "--no-other-configs"]
        keep = ("value", "ms_per_step", "step_kernel_ms", "launch_ms", "roofline", "command", "run_s", "error")
        for cfg in ("c2", "c3", "c5"):
            r = child(cfg, quick)
            k200 = {k: r[k] for k in keep if k in r}
            if cfg == "c3":
                res["c3_k200"] = k200
            else:
                res[cfg]["k200"] = k200
    return res


def main_c1(a, json_fd):
    """BASELINE config c1: one JNIBotClient env (bot-only JNIGridnetVecClient, :157-177 / JNIBotClient
    :108-135), RandomBiasedAI vs RandomBiasedAI — plumbing; the CPU oracle's rate is the reference
    figure.  GPU: the same env as a bot-only DeviceVecEnv, K steps captured in one hipGraph."""
    import torch

    from microrts_amd import DeviceVecEnv

    assert a.gpus == 1, "c1 is a one-env configuration"
    torch.cuda.set_device(0)
    env = DeviceVecEnv(0, 1, 2000, [os.path.join(ROOT, a.map)], ai1s=["RandomBiasedAI"], ai2s=["RandomBiasedAI"],
                       seed=42, with_masks=False)
    env.reset()
    for _ in range(a.burnin):
        env.step()
    graph = torch.cuda.CUDAGraph()
    cap = torch.cuda.Stream(env.device)
    cap.wait_stream(torch.cuda.current_stream(env.device))
    with torch.cuda.graph(graph, stream=cap):
        for _ in range(a.steps):
            env.step()
    torch.cuda.synchronize()
    graph.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    graph.replay()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    assert not env.error_flags().any()
    out = {
        "metric": METRIC, "value": a.steps / t, "unit": "env-steps/s", "n_gpus": 1, "rccl_world_size": 1,
        "steps": a.steps, "warmup": a.warmup, "ms_per_step": 1e3 * t / a.steps, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "int32",
        "data": "synthetic (RandomBiasedAI x 2, per-game java.util.Random seeded from 42)",
        "config": {"workload": f"c1: {a.map}, 1 env, RandomBiasedAI vs RandomBiasedAI (bot-only client, reward/done "
                               "only) — one wave on the GPU: launch latency, not throughput",
                   "burnin_steps": a.burnin, "launch": "hipGraph replay of the K timed steps",
                   "parallelism": "single env"},
    }
    if not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline_c1(os.path.join(ROOT, a.map))
    sys.stdout.flush()
    os.write(json_fd, (json.dumps(out) + "\n").encode())
    env.close()


def main():
    a = parse()
    # --gpus N without a launcher: spawn the N ranks here, before anything touches a GPU (the parent
    # only waits; each child is one rank with RANK / LOCAL_RANK / WORLD_SIZE set, as
    # torch.distributed.run would); under a launcher WORLD_SIZE must equal --gpus
    from microrts_amd.launch import check_world, free_port, spawn_ranks

    if a.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(spawn_ranks(a.gpus, [sys.executable, os.path.abspath(__file__)] + sys.argv[1:]))
    world = check_world(a.gpus)
    # stdout carries exactly one JSON line (rank 0): everything else that writes to fd 1 — RCCL's
    # version banner, library prints — goes to stderr
    json_fd = os.dup(1)
    os.dup2(2, 1)
    if a.config == "c1":
        return main_c1(a, json_fd)
    import numpy as np
    import torch
    import torch.distributed as dist

    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    # a process group always: RCCL over xGMI between the ranks, and at N = 1 a one-rank group for the
    # with-exchange window (SURVEY.md §8e's second curve)
    pg_error = None
    if world == 1 and "MASTER_PORT" not in os.environ:
        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(free_port()), RANK="0", WORLD_SIZE="1")
    try:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local), rank=rank, world_size=world)
    except Exception as ex:  # only tolerated at N = 1 (then no exchange window)
        if world > 1:
            raise
        pg_error = repr(ex)
        print(f"bench: no process group at N=1 ({pg_error}); the exchange window is skipped", file=sys.stderr)
    use_pg = dist.is_initialized()
    rccl_world = dist.get_world_size() if use_pg else 1
    assert rccl_world == world, f"process group has {rccl_world} ranks, --gpus {a.gpus}"
    from microrts_amd import DeviceVecEnv, UnitTypeTable
    from microrts_amd import dist as mdist

    E = a.envs
    utt = UnitTypeTable(a.utt, 1)
    utt_name = {1: "VERSION_ORIGINAL", 2: "VERSION_ORIGINAL_FINETUNED"}[a.utt] + ", CANCEL_BOTH"
    sh = mdist.shard(rank, E)
    env = DeviceVecEnv(sh["n_slots"], 0, 2000, [os.path.join(ROOT, a.map)] * sh["n_slots"], device=local, seed=SEED,
                       partial_obs=a.po, max_units=a.max_units, utt=utt,
                       slot_id_base=sh["slot_id_base"], mask_delta=a.mask_mode == "delta",
                       source_bits=a.mask_mode == "delta")
    S, H, W, C, K = env.dims
    stream = torch.cuda.current_stream(env.device)
    gather_buf = None
    if a.gather_obs and use_pg:
        gather_buf = mdist.ObservationGather(env.obs.shape, env.device, mode=a.gather_obs)
    xg = {"buf": gather_buf}  # the exchange one_step performs (None: no collective in the step)

    fused = a.policy == "fused"
    uniform = a.policy in ("uniform", "uniform-split")
    mode = {"fused": fused, "uni_fused": a.policy == "uniform"}

    # the exchange's int16 transport written by the step kernel itself (full observability: no
    # narrowing pass); partially observable views keep the narrowing copy in push()
    kernel16 = gather_buf is not None and not gather_buf.gloo and not a.po

    def one_step(k, ev=None):
        gather_buf = xg["buf"]
        kernel16 = gather_buf is not None and not gather_buf.gloo and not a.po
        if kernel16:
            env.set_obs16(gather_buf.begin())
        fused = mode["fused"]
        if uniform and mode["uni_fused"]:  # one launch: rows drawn and written by the step kernel
            if ev is not None:
                ev[0].record(torch.cuda.current_stream(env.device))
            env.step_uniform(SEED, k)
            if ev is not None:
                ev[1].record(torch.cuda.current_stream(env.device))
            if gather_buf is not None:
                gather_buf.finish() if kernel16 else gather_buf.push(env.obs)
            return
        if uniform:
            env.uniform_policy(SEED, k)
        elif not fused:
            env.random_policy(SEED, k)
        if ev is not None:
            ev[0].record(torch.cuda.current_stream(env.device))
        if fused:
            env.step_fused(SEED, k + 1)  # consumes the actions of step k, writes those of step k + 1
        elif uniform:
            env.step(masks=False)  # c2: no masks
        else:
            env.step()
        if ev is not None:
            ev[1].record(torch.cuda.current_stream(env.device))
        if gather_buf is not None:
            gather_buf.finish() if kernel16 else gather_buf.push(env.obs)

    env.reset()
    if fused:
        env.random_policy(SEED, 0)
    native_path = a.launch == "native" and gather_buf is None

    def run_steps(first, n):  # steps first .. first + n - 1, through the timed window's own path
        if native_path and uniform:
            env.rollout_uniform(SEED, first, n, fused=mode["uni_fused"])
        elif native_path:
            env.rollout_fused(SEED, first + 1, n)
        else:
            for k in range(first, first + n):
                one_step(k)

    run_steps(0, a.burnin)
    env.synchronize()
    # rows decoded per step (sum of mask[...,0]) and live units, for the algorithmic-byte count —
    # taken after the burn-in, so that the warmup steps run right before the timed window (no host
    # work leaves the GPU idle in between)
    if uniform:  # the steps write no masks: one untimed mask write to count the idle units
        env.get_masks()
        env.synchronize()
    rows = float(env.masks[..., 0].sum().item()) / S
    units = []
    for s in range(0, min(S, 64), 2):
        units.append(env.dump_state(s)[4])
    mean_units = float(np.mean(units))

    # The K timed steps are enqueued so that host launch overhead does not pace the GPU: by default
    # (fused policy) one native call, mrts_rollout_fused_dev, issues the K step launches from C++;
    # --launch graph captures them once into a hipGraph and replays it.  Same kernels, same arguments
    # either way (tests/test_gpu_parity.py::test_native_rollout_matches_fused_steps).  The native form
    # has the smallest fixed cost per window (tools/launch_overhead.py: 23 us vs 32 us for a warm
    # graph replay; a first replay costs ~20 us more), which matters at small K.  The step kernel's
    # duration comes from HIP events around each launch in an eager pass over the K steps that
    # follow (same stream, same episode phase): events cannot be timed inside the native or graph
    # window without changing it.
    base = a.burnin + a.warmup
    graph = None
    native = native_path
    if a.launch == "graph":
        try:
            assert gather_buf is None  # parse(): no torch.distributed collective is ever captured
            graph = torch.cuda.CUDAGraph()
            cap = torch.cuda.Stream(env.device)
            cap.wait_stream(torch.cuda.current_stream(env.device))
            with torch.cuda.graph(graph, stream=cap):
                for k in range(a.steps):
                    one_step(base + k)
            torch.cuda.synchronize(env.device)
        except Exception as ex:  # capture unsupported here: time eagerly instead
            print(f"bench: hipGraph capture failed ({ex!r}); eager launches", file=sys.stderr)
            graph = None
    try:
        evs = [(_FenceFreeEvent(), _FenceFreeEvent()) for _ in range(a.steps)]
        event_kind = "hipEventDisableSystemFence events"
    except (OSError, AttributeError) as ex:
        print(f"bench: fence-free events unavailable ({ex!r}); torch.cuda.Event", file=sys.stderr)
        evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(a.steps)]
        event_kind = "torch.cuda.Event"
    # multi-step launches: the native fused rollout runs the K steps of every game in one k_env launch
    # (state in LDS between steps; mrts_rollout_fused_dev), so the launch's own duration is the
    # kernel time — fence-free events around it inside the timed window
    multi = native and ((fused and env.fused_multi_step) or (uniform and mode["uni_fused"] and env.multi_step_capable))
    roll_ev = (_FenceFreeEvent(), _FenceFreeEvent()) if multi and event_kind.startswith("hipEvent") else None
    if roll_ev is not None and a.warmup > 0:
        # the warmup launch carries events too: the first event-carrying dispatch of a process pays a
        # one-time runtime cost (~15 us), which belongs to the warmup, not to the window
        warm_ev = (_FenceFreeEvent(), _FenceFreeEvent())
        env.set_rollout_events(warm_ev[0].h, warm_ev[1].h)
    run_steps(a.burnin, a.warmup)  # the W untimed warmup steps, immediately before the window
    if roll_ev is not None:  # the library records them around the window's launch (mrts_set_rollout_events)
        env.set_rollout_events(roll_ev[0].h, roll_ev[1].h)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(env.device)
    env.synchronize()
    t0 = time.perf_counter()
    if native and uniform:
        env.rollout_uniform(SEED, base, a.steps, fused=mode["uni_fused"])
    elif native:
        env.rollout_fused(SEED, base + 1, a.steps)
    elif graph is not None:
        graph.replay()
    else:
        for k in range(a.steps):
            one_step(base + k, evs[k])
    if gather_buf is not None:
        gather_buf.wait()  # the last step's exchange belongs to the timed window
    torch.cuda.synchronize(env.device)  # device-wide: covers the env's stream too
    if world > 1:
        dist.barrier()
    t = time.perf_counter() - t0
    if native or graph is not None:  # kernel-duration pass (untimed for `value`)
        # hold the stream in a GPU spin while the host enqueues the K eager steps, so each event
        # pair brackets back-to-back kernels instead of the host's launch latency
        try:
            torch.cuda._sleep(int(150_000 * a.steps))
        except (AttributeError, RuntimeError):
            pass
        for k in range(a.steps):
            one_step(base + a.steps + k, evs[k])
        torch.cuda.synchronize(env.device)
        base += a.steps
    t = mdist.max_over_ranks(t, env.device)
    step_ms = [s.elapsed_time(e) for s, e in evs]
    kern_ms = float(np.mean(step_ms))
    single_kern_ms = kern_ms  # one step per launch (the eager event pass)
    launch_ms = None
    if roll_ev is not None:  # the multi-step launch: its duration / K is the per-step kernel time
        launch_ms = roll_ev[0].elapsed_time(roll_ev[1])
        kern_ms = launch_ms / a.steps
    flags = env.error_flags()
    assert not flags.any(), f"engine error flags set: {np.unique(flags)}"

    # Roofline bytes per step-kernel launch.  The step's HBM contract under the persistent-buffer
    # (delta) mask mode — what any implementation must move:
    #   A = idle-unit action rows read (28 B each; other rows are ignored by the Java decode; 4 B when
    #       the fused policy forwards them),
    #   O = C*HW*4 observation written per slot,
    #   M = K bytes per mask row that changed (delta) or HW*K per slot (full rewrite),
    #   S = per game: header 64 B + 28 B/unit, read and written; terrain HW B read; previous row sets
    #       (2 * maskWords * 4 B) read and written; per slot the source bits (maskWords * 4 B) written.
    # SURVEY.md §8(d)'s figure assumed a full mask rewrite and all rows read; it is reported next to it.
    HW = H * W
    MWB = 0 if uniform else 4 * ((HW + 31) // 32)  # mask row sets / source bits: only with masks
    dirty = rows
    # partially observable views under the persistent-buffer contract (DeviceVecEnv obs_delta): only
    # the (plane, 4-cell chunk) pieces that changed must be written — measured on the probe steps
    po_delta = a.po and (HW % 4) == 0 and W <= 32 and H <= 32
    obs_chunks = float(C * HW // 4)
    if env.source is not None and a.mask_mode == "delta" and not uniform:
        lut = torch.tensor([bin(i).count("1") for i in range(256)], dtype=torch.int64, device=env.device)
        tot, otot, n_probe = 0, 0, 5
        for k in range(n_probe):  # untimed probe steps after the timed window
            before = env.source.clone()
            obefore = env.obs.clone() if po_delta else None
            one_step(base + a.steps + k)  # after the timed (and kernel-timing) windows
            env.synchronize()
            tot += int(lut[(before | env.source).view(torch.uint8).long()].sum().item())
            if po_delta:
                otot += int((obefore != env.obs).view(S, C, HW // 4, 4).any(-1).sum().item())
        dirty = tot / (n_probe * S)
        if po_delta:
            obs_chunks = otot / (n_probe * S)
    n_games = S // 2
    m_bytes = 0 if uniform else (dirty * K if a.mask_mode == "delta" else HW * K)
    o_bytes = obs_chunks * 16  # C * HW * 4 for a full write
    if launch_ms is not None and not a.po:  # a multi-step launch stores the static terrain plane once
        o_bytes = (C - 1) * HW * 4 + HW * 4 / a.steps
    # fused policy: the idle units' rows arrive as one forwarded 4-B word each (KDyn.fwd_read), and the
    # step writes that word next to the 28-B row it leaves in the action tensor
    # fused uniform policy: no row is read (the idle units' rows are drawn in registers), and every row
    # of the action tensor is written by the step kernel
    uni_fused = uniform and mode["uni_fused"]
    row_in = 4 if fused else 0 if uni_fused else 28
    # per game: the state (header + unit rows) read and written, the terrain read, both players' row sets
    # read and written — per step; a multi-step launch keeps state, terrain, row sets and forwarded
    # words in LDS / registers, so it loads them at its first step and stores them after its last
    # (1/K per step)
    state_io = 2 * (64 + 28 * mean_units) + HW
    multi_l = launch_ms is not None
    if multi_l:
        row_in = row_in / a.steps if fused else row_in
        contract = S * (rows * row_in + o_bytes + m_bytes + MWB) + n_games * (state_io + 2 * 2 * MWB) / a.steps
    else:
        contract = S * (rows * row_in + o_bytes + m_bytes + MWB) + n_games * (state_io + 2 * 2 * MWB)
    if fused:  # the policy's action rows (and their forwarded words) leave the step kernel too
        contract += S * (dirty if a.mask_mode == "delta" else HW) * 28 + S * rows * 4 / (a.steps if multi_l else 1)
    if uni_fused:
        contract += S * HW * 28
    survey = S * (HW * 7 * 4 + C * HW * 4 + (0 if uniform else HW * K) + (16 * mean_units + 2 * HW + 16))
    achieved = contract / (kern_ms * 1e-3) / 1e9
    # a launch = the K steps of the multi-step launch, else one step
    steps_per_launch = a.steps if launch_ms is not None else 1
    # roofline.traffic: HBM bytes per k_env launch from the rocprofv3 --pmc passes of this same command
    # (tools/gpu_profile.sh + tools/summarize_profile.py -> profiles/pmc_latest.json), when they exist
    traffic, traffic_src = a.pmc_traffic, "--pmc-traffic (bytes per launch)" if a.pmc_traffic is not None else None
    # per-config counters of the same command (tools/profile_config.sh + tools/profile_summary.py)
    pj = None
    pmc_note = None
    pl = os.path.join(ROOT, "profiles", f"pmc_{a.config}.json")
    if os.path.exists(pl):
        pj = json.load(open(pl))
        if not (pj.get("envs_per_gpu") == E and a.map in (pj.get("workload") or "")
                and pj.get("utt", "VERSION_ORIGINAL, CANCEL_BOTH") == utt_name
                and pj.get("mask_mode") == ("off" if uniform else a.mask_mode) and launch_ms is not None):
            pj = None  # another workload or launch form: its counters do not describe this line
        elif pj.get("gfx950_code_sha256") != code_sha256():
            pmc_note = (f"profiles/pmc_{a.config}.json was taken with other kernel code "
                        f"({(pj.get('gfx950_code_sha256') or 'no hash')[:12]}); its counters are not used")
            pj = None  # stale counters must not describe this library's kernel
    if traffic is None and pj is not None and pj.get("traffic_bytes_per_step"):
        per_step = pj["traffic_bytes_per_step"]
        traffic = per_step * steps_per_launch
        traffic_src = (f"profiles/pmc_{a.config}.json ({pj['tag']}: 2 x FETCH_SIZE + WRITE_SIZE, separate --pmc passes; "
                       f"{per_step / 1e6:.1f} MB per step x {steps_per_launch} steps per launch)")
    issue = None
    if pj is not None and pj.get("issue"):
        # The issue roofline: VALU instructions per game-step (SQ_INSTS_VALU, this library's
        # PMC pass) x game-steps/s against the SIMDs' VALU issue ceiling for THIS kernel's instruction mix:
        # 1024 SIMDs x clock / c_mix, c_mix = the cycles per wave64 VALU instruction that the issue probe
        # (tools/probes/valu_issue_probe.hip) measures per opcode class at the kernel's waves per SIMD with
        # full EXEC, weighted by the kernel's static VALU opcode mix (tools/issue_roofline.py ->
        # profiles/issue_ceiling_<cfg>.json).  The guide's flat 2 cycles per instruction is reported beside it.
        iq = pj["issue"]
        per = iq["per_game_step"]
        clk = iq.get("clock_ghz_grbm") or 2.4
        rate = E / (kern_ms * 1e-3)  # game-steps per second of kernel time
        valu = per["SQ_INSTS_VALU"] * rate
        icp = os.path.join(ROOT, "profiles", f"issue_ceiling_{a.config}.json")
        ic = json.load(open(icp)) if os.path.exists(icp) else None
        c_mix = ic["c_mix_cycles"] if ic else 2.0
        ceiling = 1024 * clk * 1e9 / c_mix
        issue = {
            "achieved": valu / 1e9,
            "peak": ceiling / 1e9,
            "unit": "G wave64 VALU instructions/s",
            "frac": valu / ceiling,
            "c_mix_cycles_per_valu": c_mix,
            "cycles_per_valu_achieved": 1024 * clk * 1e9 / valu,
            "frac_vs_guide_2_cycles": valu / (1024 * clk * 1e9 / 2),
            "valu_insts_per_game_step": per["SQ_INSTS_VALU"],
            "salu_insts_per_game_step": per.get("SQ_INSTS_SALU"),
            "lds_insts_per_game_step": per.get("SQ_INSTS_LDS"),
            "valu_lane_utilization": iq.get("valu_lane_utilization"),
            "valu_busy_frac": iq.get("valu_busy_frac"),
            "dual_issue_quad_cycles_per_game_step": per.get("SQ_ACTIVE_INST_VALU2"),
            "clock_ghz": clk,
            "games_per_simd": iq.get("games_per_simd"),
            "source": f"profiles/pmc_{a.config}.json ({pj['tag']}: SQ PMC pass of the same command, same gfx950 code object) + "
                      + (f"profiles/issue_ceiling_{a.config}.json (probe {ic['probe']}, static mix of {ic['static_valu_instructions']} "
                         "VALU opcodes)" if ic else "no issue_ceiling file: the guide's 2 cycles"),
        }
    hbm_frac = achieved / HBM_PEAK_GBS
    # what the numbers show bounds the kernel: VALU issue when the SIMDs issue this mix near its measured
    # ceiling (c3: four games per SIMD), else the per-game dependent chain (c2 / c5: one / two games per
    # SIMD leave issue slots idle); HBM only without counters
    if issue is not None and issue["frac"] >= 0.6 and issue["frac"] > hbm_frac:
        bound, bound_note = "valu_issue", ("VALU issue at {:.2f} of this kernel's probe-measured ceiling ({:.2f} cycles per "
                                           "instruction for its mix; achieved {:.2f}), HBM at {:.2f} of peak (step-contract "
                                           "bytes, roofline.frac)".format(issue["frac"], issue["c_mix_cycles_per_valu"],
                                                                          issue["cycles_per_valu_achieved"], hbm_frac))
    elif issue is not None:
        bound, bound_note = "latency", ("per-game dependent chain: VALU issue at {:.2f} of the probe-measured ceiling with "
                                        "{:.0f} game(s) per SIMD (roofline.issue); HBM at {:.2f} of peak (step-contract "
                                        "bytes)".format(issue["frac"], issue.get("games_per_simd") or 0, hbm_frac))
    else:
        bound, bound_note = "hbm", "HBM step-contract bytes (no counter file of this library for this workload)"
    total_games = E * world
    value = total_games * a.steps / t
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "rccl_world_size": rccl_world,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": 1e3 * t / a.steps,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int32",
        "data": ("synthetic (unmasked uniform random rows for every cell, Philox seed 0x5EEDC0DE)" if uniform
                 else "synthetic (masked uniform random policy, Philox seed 0x5EEDC0DE)"),
        "parity": "bit-exact: the reference's 280 recorded games (data/traces, 17,085 entries) replay through these HIP "
                  "kernels with every PhysicalGameState equal to the trace's (tests/test_gpu_traces.py); every output vs the "
                  "trace-pinned C++ oracle (tests/test_gpu_parity.py, test_headline_parity.py at this config's full size, "
                  "test_kats.py); Java itself cannot run in this image",
        "config": {
            "workload": f"{a.config}: {a.map} self-play, {E} games/GPU ({2 * E} player slots), "
                        + ("obs every step, no masks (SURVEY §8(d) c2)" if uniform else "masks+obs every step")
                        + (", partial observability" if a.po else "")
                        + (f", max_units {a.max_units} (capacity errors checked)" if a.max_units else "")
                        + (f", UTT version {a.utt}" if a.utt != 1 else ""),
            "envs_per_gpu": E,
            "utt": utt_name,
            "reward_functions": "[WinLossRewardFunction] (with one reward function Java's self-play reset throws, "
                                "JNIGridnetClientSelfPlay.java:235-238; here the one slot is zeroed — DESIGN.md §8)",
            "max_steps": 2000,
            "burnin_steps": a.burnin,
            "mask_mode": "off" if uniform else a.mask_mode,
            "launch": (f"one {'mrts_rollout_uniform_dev' if uniform else 'mrts_rollout_fused_dev'} call: ONE k_env launch runs the K steps of every game (multi-step "
                       "launch, each game's state kept in LDS between its steps; every step's observation, masks, "
                       "rewards, dones and next action rows written to HBM)" if multi
                       else "one mrts_rollout_uniform_dev call (K fused policy+step launches from C++)" if native and uni_fused
                       else "one mrts_rollout_uniform_dev call (K policy + K step launches from C++)" if native and uniform
                       else "one mrts_rollout_fused_dev call (K step launches from C++)" if native
                       else "hipGraph replay of the K timed steps" if graph is not None else "eager"),
            "policy": ("unmasked uniform rows drawn and written by the step kernel (mrts_step_uniform_dev, "
                       "bit-identical to a policy launch + a step launch)" if uni_fused
                       else "unmasked uniform rows, separate kernel before each step (mrts_policy_uniform_dev, inside the "
                       "timed window)" if uniform
                       else "fused into the step kernel (mrts_step_fused_dev)" if fused
                       else "separate masked-uniform policy kernel before each step (mrts_policy_dev)"),
            "kernel_timing": (f"{event_kind} recorded by the multi-step launch's own dispatch in the timed window "
                              "(mrts_set_rollout_events: hipExtLaunchKernelGGL start / stop events), / K" if launch_ms is not None
                              else f"{event_kind} around each step-kernel launch, eager pass over the next K steps"
                              if (native or graph is not None) else f"{event_kind} around each step-kernel launch in the timed window"),
            "parallelism": f"dp{world} (independent env shards)" + (
                f", per-step RCCL int16 observation {a.gather_obs} overlapped on a comm stream"
                + (" (int16 transport written by the step kernel)" if kernel16 else "") if gather_buf is not None
                else ", no collective in the step"),
        },
        "step_kernel_ms": kern_ms,
        "launch_ms": launch_ms,
        "single_step_launch_kernel_ms": single_kern_ms,
        "mean_units": mean_units,
        "decoded_rows_per_slot": rows,
        "roofline": {
            "bound": bound,
            "bound_note": bound_note,
            "issue": issue,
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": traffic,
            "traffic_source": traffic_src if pmc_note is None else pmc_note,
            "kernel": "k_env<MODE_STEP>" + (" + fused policy rows" if fused else " + fused uniform rows" if uni_fused else ""),
            "alg_bytes_per_launch": contract * steps_per_launch,
            "alg_bytes_per_step": contract,
            "launch_duration_ms": kern_ms * steps_per_launch,
            "alg_bytes_note": f"step contract bytes, {'no' if uniform else a.mask_mode} masks: {rows:.2f} idle-unit rows and {dirty:.2f} "
                              f"changed mask rows per slot" + (f", {obs_chunks:.1f} changed (plane, 4-cell chunk) "
                              f"observation pieces per slot (persistent PO views)" if po_delta else "")
                              + " (DESIGN.md §5)",
            "survey_8d_bytes_per_launch": survey,
            "survey_8d_equivalent_GBps": survey / (kern_ms * 1e-3) / 1e9,
        },
    }
    if traffic:
        # the PMC bytes against the contract: below it, the outputs rewritten every step stay in L2 / MALL between
        # launches (c2: 1024 games' planes), so frac is a fraction of the contract's bytes, not of HBM bytes moved
        rf = out["roofline"]
        rf["traffic_GBps"] = traffic / (kern_ms * steps_per_launch * 1e-3) / 1e9
        rf["traffic_frac"] = rf["traffic_GBps"] / HBM_PEAK_GBS
        rf["traffic_over_contract"] = traffic / (contract * steps_per_launch)
        rf["frac_basis"] = ("contract bytes (L2-resident: the PMC-measured HBM traffic is {:.2f} of the contract, so the "
                            "HBM fraction actually moved is traffic_frac)".format(rf["traffic_over_contract"])
                            if rf["traffic_over_contract"] < 0.8 else "contract bytes (PMC traffic {:.2f} of them)"
                            .format(rf["traffic_over_contract"]))
    if world == 1 and (native or graph is not None) and gather_buf is None and not a.no_compare and not uniform:
        # the other policy form over the next K steps, for comparison (same contract otherwise)
        mode["fused"] = not fused
        base2 = base + a.steps + 5
        if mode["fused"]:
            env.random_policy(SEED, base2)
        g2 = torch.cuda.CUDAGraph()
        cap = torch.cuda.Stream(env.device)
        cap.wait_stream(torch.cuda.current_stream(env.device))
        with torch.cuda.graph(g2, stream=cap):
            for k in range(a.steps):
                one_step(base2 + k)
        torch.cuda.synchronize(env.device)
        t1 = time.perf_counter()
        g2.replay()
        torch.cuda.synchronize(env.device)
        t2 = time.perf_counter() - t1
        out["other_policy_form"] = {"policy": "fused" if mode["fused"] else "kernel", "value": total_games * a.steps / t2,
                                    "ms_per_step": 1e3 * t2 / a.steps}
        mode["fused"] = fused
        assert not env.error_flags().any()
    if world == 1 and multi and not a.no_compare:
        # the same native rollout with one launch per step (mrts_set_multi_step(0)), next K steps
        base3 = base + 2 * a.steps + 10
        env.set_multi_step(False)
        roll = (lambda f, n: env.rollout_uniform(SEED, f, n)) if uniform else (lambda f, n: env.rollout_fused(SEED, f, n))
        roll(base3 - 4, 5)
        torch.cuda.synchronize(env.device)
        t1 = time.perf_counter()
        roll(base3 + 1, a.steps)
        torch.cuda.synchronize(env.device)
        t2 = time.perf_counter() - t1
        env.set_multi_step(True)
        out["single_step_launches"] = {"value": total_games * a.steps / t2, "ms_per_step": 1e3 * t2 / a.steps,
                                       "step_kernel_ms": single_kern_ms,
                                       "launch": f"one {'mrts_rollout_uniform_dev' if uniform else 'mrts_rollout_fused_dev'} "
                                                 "call issuing K single-step launches"}
        assert not env.error_flags().any()
    if world == 1 and native and uniform and gather_buf is None and not a.no_compare:
        # the other uniform form (fused <-> split) over the next K steps, native launches both
        base2 = base + a.steps + 5
        env.rollout_uniform(SEED, base2 - 5, 5, fused=not mode["uni_fused"])
        torch.cuda.synchronize(env.device)
        t1 = time.perf_counter()
        env.rollout_uniform(SEED, base2, a.steps, fused=not mode["uni_fused"])
        torch.cuda.synchronize(env.device)
        t2 = time.perf_counter() - t1
        out["other_policy_form"] = {"policy": "uniform-split" if mode["uni_fused"] else "uniform",
                                    "value": total_games * a.steps / t2, "ms_per_step": 1e3 * t2 / a.steps}
        assert not env.error_flags().any()
    if not a.no_full_contract and not uniform and gather_buf is None:
        out["full_contract"] = full_contract_window(a, sh, local, base, E * world, world, mdist, torch, dist, DeviceVecEnv)
    if gather_buf is None and not a.no_gather_window:
        # SURVEY.md §8e's second curve: the same steps with the north-star observation exchange — by
        # default the compact game records of every step, all-gathered once per launch (records_window,
        # DESIGN.md §7); --gather-window tensor: the per-step all-gather of the observation tensor itself
        # (one step launch per step, libmrts's own capture of the steps and their collectives).
        if not use_pg:
            out["with_gather"] = {"error": f"no process group: {pg_error}"}
        else:
            def give_up():  # a collective that never completes (the exchange has no other way out)
                print(f"bench: exchange window exceeded {a.gather_timeout:.0f} s; giving it up", file=sys.stderr)
                if rank == 0:
                    out["with_gather"] = {"error": f"timed out after {a.gather_timeout:.0f} s"}
                    sys.stdout.flush()
                    os.write(json_fd, (json.dumps(out) + "\n").encode())
                sys.stderr.flush()
                os._exit(0)

            records_ok = (a.gather_window == "records" and dist.get_backend() != "gloo" and native
                          and (mode["fused"] or mode["uni_fused"]))
            try:
                if records_ok:
                    out["with_gather"] = run_with_deadline(
                        lambda: records_window(env, a, mode, base + 3 * a.steps + 20, E * world, world, mdist, torch, dist),
                        a.gather_timeout, give_up)
                else:
                    out["with_gather"] = run_with_deadline(
                        lambda: gather_window(env, a, xg, one_step, base + 3 * a.steps + 20, E * world, world, mdist, torch,
                                              dist, mode), a.gather_timeout, give_up)
            except Exception as ex:  # the headline line must survive a failed exchange window
                print(f"bench: exchange window failed: {ex!r}", file=sys.stderr)
                out["with_gather"] = {"error": repr(ex)}
            assert not env.error_flags().any()
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(os.path.join(ROOT, a.map), a.cpu_threads or all_cores(), a.burnin, uniform, po=a.po,
                                           utt=a.utt)
    env.close()
    if use_pg:
        dist.destroy_process_group()
    if rank == 0 and world == 1 and a.config == "c3" and not a.no_other_configs and a.utt == 1 and a.envs == CONFIGS["c3"][1]:
        out["configs"] = other_configs(a)
    if rank == 0:
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(out) + "\n").encode())


if __name__ == "__main__":
    main()
