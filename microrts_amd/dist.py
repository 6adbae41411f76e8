"""Multi-GPU plumbing for the env step: one process per GPU, disjoint game shards,
no collective inside the step.  Backend-agnostic (RCCL on MI355X, gloo on CPU for the tests)."""
import torch
import torch.distributed as dist


def shard(rank, games_per_rank):
    """Slots of rank r are global slots [r*2G, (r+1)*2G): self-play game g of rank r is global game
    r*G + g.  slot_id_base feeds every per-slot RNG stream (Philox policy counter, java.util.Random
    seeds), so the shards never share a stream and N ranks reproduce one N*G-game run."""
    return {"slot_id_base": rank * 2 * games_per_rank, "n_slots": 2 * games_per_rank}


def max_over_ranks(seconds, device):
    """The job's time = the slowest rank's (bench.py contract)."""
    if not dist.is_initialized() or dist.get_world_size() == 1:
        return seconds
    t = torch.tensor([seconds], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_observations(obs, out=None, transport=torch.int16):
    """North-star RCCL all-gather of the batched observation tensor (int16 transport: every plane
    value fits — hp <= 10, resources <= 32767 by map validation).  Returns [world, *obs.shape]."""
    world = dist.get_world_size()
    if dist.get_backend() == "gloo":
        transport = torch.int32  # gloo has no int16 collectives
    send = obs.to(transport).contiguous()
    if out is None:
        out = torch.empty((world,) + tuple(obs.shape), dtype=transport, device=obs.device)
    if dist.get_backend() == "gloo":
        dist.all_gather(list(out.unbind(0)), send)
    else:  # RCCL/NCCL has no int16 type: move the same bytes as float16 (a gather does no arithmetic)
        dist.all_gather_into_tensor(_wire(out.view(-1)), _wire(send.view(-1)))
    return out


def _wire(t):
    return t.view(torch.float16) if t.dtype == torch.int16 else t


class ObservationGather:
    """The north-star observation exchange of every step, overlapped with the next
    step's compute: the observation of step t is narrowed to the int16 transport (hp <= 10,
    resources <= 32767 by map validation) into buffer t % 2 on the compute stream, and a separate
    communication stream runs the collective while step t+1 computes; buffer t % 2 is reused only
    after the collective of step t-2 finished.

    mode "allgather": every rank receives [world, *obs.shape] (RCCL all-gather, ring, per-link bound);
    mode "learner": only rank 0 receives it (gather to one rank: each peer sends once on its own
    link).  gloo (the CPU tests) has no int16 collectives and no streams: int32, synchronous."""

    def __init__(self, obs_shape, device, mode="allgather"):
        if mode not in ("allgather", "learner"):
            raise ValueError("mode must be 'allgather' or 'learner'")
        self.mode = mode
        self.world, self.rank = dist.get_world_size(), dist.get_rank()
        self.gloo = dist.get_backend() == "gloo"
        self.transport = torch.int32 if self.gloo else torch.int16
        shape = tuple(obs_shape)
        self.send = [torch.empty(shape, dtype=self.transport, device=device) for _ in range(2)]
        recv = mode == "allgather" or self.rank == 0
        self.recv = [torch.empty((self.world,) + shape, dtype=self.transport, device=device) if recv else None
                     for _ in range(2)]
        cuda = device.type == "cuda" and not self.gloo
        self.comm = torch.cuda.Stream(device) if cuda else None
        self.done = [torch.cuda.Event() for _ in range(2)] if cuda else None
        self.fired = [False, False]
        self.i = 0

    def _collective(self, b):
        # RCCL has no int16 collectives: the int16 buffers travel as float16 views (pure byte moves)
        send = _wire(self.send[b])
        if self.mode == "allgather":
            if self.gloo:
                dist.all_gather(list(self.recv[b].unbind(0)), self.send[b])
            else:
                dist.all_gather_into_tensor(_wire(self.recv[b]).view(-1), send.view(-1))
        else:
            recv = [_wire(x) for x in self.recv[b].unbind(0)] if self.rank == 0 else None
            dist.gather(send, gather_list=recv, dst=0)

    def push(self, obs):
        """Call after the step that produced `obs`, on the compute stream.  Returns the receive
        buffer of this step (None on non-learner ranks in "learner" mode); it is complete after
        wait() or once the next-but-one push() returned."""
        b = self.i & 1
        self.i += 1
        if self.comm is None:
            self.send[b].copy_(obs)
            self._collective(b)
            return self.recv[b]
        cur = torch.cuda.current_stream(obs.device)
        if self.fired[b]:
            cur.wait_event(self.done[b])  # buffer b still feeds the collective of two steps ago
        self.send[b].copy_(obs)
        ready = torch.cuda.Event()
        ready.record(cur)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ready)
            self._collective(b)
            self.done[b].record(self.comm)
        self.fired[b] = True
        return self.recv[b]

    def begin(self):
        """Kernel-written transport (DeviceVecEnv.set_obs16): the int16 send buffer the NEXT step
        must write, after making the current stream wait until the collective that last read it
        (two steps ago) finished.  Pass it to env.set_obs16, run the step, then call finish()."""
        b = self.i & 1
        if self.comm is not None and self.fired[b]:
            torch.cuda.current_stream(self.send[b].device).wait_event(self.done[b])
        return self.send[b]

    def finish(self):
        """The step that wrote begin()'s buffer is enqueued: start its collective (as push(), without
        the narrowing copy).  Returns this step's receive buffer (None on non-learner ranks)."""
        b = self.i & 1
        self.i += 1
        if self.comm is None:
            self._collective(b)
            return self.recv[b]
        cur = torch.cuda.current_stream(self.send[b].device)
        ready = torch.cuda.Event()
        ready.record(cur)
        with torch.cuda.stream(self.comm):
            self.comm.wait_event(ready)
            self._collective(b)
            self.done[b].record(self.comm)
        self.fired[b] = True
        return self.recv[b]

    def wait(self):
        """Make the current stream wait for every collective issued so far."""
        if self.comm is not None:
            cur = torch.cuda.current_stream(self.send[0].device)
            for b in range(2):
                if self.fired[b]:
                    cur.wait_event(self.done[b])


def rccl_library_path():
    """The RCCL library this process loaded (torch's process group uses it; the native exchange takes
    its entry points from the same instance), or "librccl.so" when none is mapped yet."""
    import os

    with open("/proc/self/maps") as f:
        for line in f:
            if "librccl.so" in line:
                return line.split()[-1]
    bundled = os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")
    return bundled if os.path.exists(bundled) else "librccl.so"


class NativeExchange:
    """The observation exchange of every step from native code (mrts_rollout_*_exchange_dev): one RCCL
    communicator per rank's handle (its unique id broadcast over the torch process group), the step
    kernel writing the int16 transport into send buffer t % 2, the all-gather of step t on the
    handle's own stream overlapping step t + 1, no Python between steps and no graph capture.  Full
    observability; every rank of `group` must construct it (ncclCommInitRank is collective)."""

    def __init__(self, env, group=None, u8=False):
        """u8: exchange the observation as uint8 (mrts_set_exchange_bytes: half the bytes) when the
        handle allows it (16x16 full observability, every value < 256), else int16; "auto" = try.
        Every rank decides the same way (the handles are built alike)."""
        import ctypes

        from microrts_amd import _lib

        self.env = env
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        L, h = env._h.L, env._h.h
        path = rccl_library_path().encode()
        uid = (ctypes.c_char * 128)()
        # every rank binds RCCL first (drawing an id it may not use) and the ranks agree before anyone
        # enters the collective init: a rank that failed alone would leave the others waiting in it
        ok = L.mrts_rccl_unique_id(path, uid) == 0
        flag = torch.tensor([1 if ok else 0], device=env.device if dist.get_backend(group) != "gloo" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if not bool(flag.item()):
            why = L.mrts_last_error().decode() if not ok else "another rank"
            raise RuntimeError(f"RCCL could not be bound on every rank: {why}")
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = (ctypes.c_char * 128).from_buffer_copy(box[0])
        _lib.check(L.mrts_exchange_init(h, path, self.world, self.rank, uid))
        self.u8 = False
        if u8:
            rc = L.mrts_set_exchange_bytes(h, 1)
            if rc != 0 and u8 != "auto":
                _lib.check(rc)
            self.u8 = rc == 0
        dt = torch.uint8 if self.u8 else torch.int16
        shape = tuple(env.obs.shape)
        self.send = [torch.zeros(shape, dtype=dt, device=env.device) for _ in range(2)]
        self.recv = torch.zeros((self.world,) + shape, dtype=dt, device=env.device)

    def rollout_fused(self, seed, first_next_step, n_steps):
        """env.rollout_fused(...) with every step's observation all-gathered into self.recv."""
        self.env.rollout_fused_exchange(seed, first_next_step, n_steps, self.send, self.recv)

    def rollout_uniform(self, seed, first_step, n_steps):
        """env.rollout_uniform(...) (fused form) with every step's observation all-gathered."""
        self.env.rollout_uniform_exchange(seed, first_step, n_steps, self.send, self.recv)

    def capture(self, fn):
        """Capture fn()'s exchange rollout calls as one graph on a side stream (env.capture: the
        collectives are this handle's own RCCL communicator, not the process group's, so no watchdog
        tracks them); replay() launches it — the same steps, verbatim, no host work per step."""
        cap = torch.cuda.Stream(self.env.device)
        cap.wait_stream(torch.cuda.current_stream(self.env.device))
        self.env.capture(fn, cap)
        torch.cuda.current_stream(self.env.device).wait_stream(cap)

    def replay(self):
        self.env.replay()


class RecordExchange:
    """The compact observation exchange (mrts_rollout_*_records_dev): every step's game
    records — the unit lists GameState.getVectorObservation reads (rts/GameState.java:922-968), ~20x
    fewer bytes than the observation planes — all-gathered over the handle's own RCCL communicator,
    one in-place all-gather per launch, overlapping the next launch; env.render_records rebuilds any
    rank's observations.  Every rank of `group` must construct it (ncclCommInitRank is collective)."""

    def __init__(self, env, units_per_record=64, steps_per_launch=0, group=None):
        import ctypes

        from microrts_amd import _lib

        self.env = env
        self.world, self.rank = dist.get_world_size(group), dist.get_rank(group)
        L, h = env._h.L, env._h.h
        self.words = env.set_records(units_per_record, steps_per_launch)
        path = rccl_library_path().encode()
        uid = (ctypes.c_char * 128)()
        ok = L.mrts_rccl_unique_id(path, uid) == 0
        flag = torch.tensor([1 if ok else 0], device=env.device if dist.get_backend(group) != "gloo" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=group)
        if not bool(flag.item()):
            why = L.mrts_last_error().decode() if not ok else "another rank"
            raise RuntimeError(f"RCCL could not be bound on every rank: {why}")
        box = [bytes(uid)]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = (ctypes.c_char * 128).from_buffer_copy(box[0])
        _lib.check(L.mrts_exchange_init(h, path, self.world, self.rank, uid))
        self.recv = None

    def buffer(self, n_steps):
        if self.recv is None or self.recv.numel() < n_steps * self.world * (self.env.dims[0] // 2) * self.words:
            self.recv = self.env.records_buffer(n_steps, self.world)
        return self.recv

    def rollout_fused(self, seed, first_next_step, n_steps):
        """env.rollout_fused(...) with every step's records all-gathered into self.recv; returns the
        per-step (offset, rank stride) table."""
        return self.env.rollout_fused_records(seed, first_next_step, n_steps, self.buffer(n_steps))

    def rollout_uniform(self, seed, first_step, n_steps):
        return self.env.rollout_uniform_records(seed, first_step, n_steps, self.buffer(n_steps))

    def render(self, offsets, step, out):
        """All ranks' observations of step `step` of the last rollout into out [world * slots, C, H, W]."""
        off, stride = offsets[step]
        return self.env.render_records(self.recv, int(off), int(stride), self.world, out)

    def check(self):
        """Raise if a rendered record was truncated (a sender's game held more units than a record, or a
        value outside its range: mrts_render_status) or one of this rank's games overflowed its record
        (MRTS_ERR_RECORD).  Synchronises; call it at a point where the learner may wait."""
        if self.env.render_overflow():
            raise RuntimeError("a rendered observation record overflowed (units missing): raise units_per_record")
        if (self.env.error_flags() & (1 << 6)).any():
            raise RuntimeError("a game of this rank overflowed its observation record (MRTS_ERR_RECORD)")
