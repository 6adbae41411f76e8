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
    else:
        dist.all_gather_into_tensor(out.view(-1), send.view(-1))
    return out
