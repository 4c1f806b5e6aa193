"""Data-parallel exchange of the PPO update over torch.distributed (RCCL on MI355X, gloo in tests).

The env step needs no collective.  The update has exactly these exchanges per minibatch:
  * the policy gradient: one flat fp32 bucket (856,972 values, 3.4 MB for the t1 policy) all-reduced and
    divided by the world size between backward() and clip_grad_norm_ (dh_ppo.py:180-181) -- one RCCL ring
    all-reduce over xGMI instead of one per parameter tensor;
  * the KL mean of the adaptive learning-rate schedule (dh_ppo.py:141-151), so every rank keeps the same lr;
and once per iteration the advantage mean / std (rollout_storage.py:119).  With equal shards these reproduce
single-process statistics of the concatenated rollout.  Single-process runs take the exact reference path.
"""
import torch
import torch.distributed as dist


def active():
    return dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1


def world():
    return dist.get_world_size() if active() else 1


def _comm_device(t):
    # RCCL works on device tensors; gloo on host tensors
    return t.device if dist.get_backend() == "nccl" else torch.device("cpu")


def all_reduce_mean_(t):
    """In-place mean over ranks (no-op in a single process)."""
    if not active():
        return t
    x = t.to(_comm_device(t))
    dist.all_reduce(x)
    x /= world()
    if x is not t:
        t.copy_(x)
    return t


def global_mean_std(x):
    """Mean and unbiased std of x over all ranks' elements (torch.mean / torch.std in a single process)."""
    if not active():
        return x.mean(), x.std()
    n = torch.tensor([float(x.numel())], dtype=torch.float64, device=x.device)
    s = x.double().sum().reshape(1)
    t = torch.cat([s, n]).to(_comm_device(x))
    dist.all_reduce(t)
    mean = (t[0] / t[1]).to(x.device)
    q = ((x.double() - mean) ** 2).sum().reshape(1).to(_comm_device(x))
    dist.all_reduce(q)
    var = q.to(x.device) / (t[1].to(x.device) - 1.0)
    return mean.to(x.dtype), var.sqrt().to(x.dtype).reshape(())


class GradientBucket:
    """Every parameter's .grad is a view into one contiguous fp32 bucket, so the gradient all-reduce (mean over
    ranks) is one collective on the bucket itself: backward() accumulates straight into it and no copy in or out
    is needed.  The owner must zero the gradients in place (optimizer.zero_grad(set_to_none=False)) so that
    autograd keeps accumulating into the views; bind_() re-attaches them if something replaced a .grad."""

    def __init__(self, params):
        self.params = [p for p in params if p.requires_grad]
        n = sum(p.numel() for p in self.params)
        dev = self.params[0].device
        self.flat = torch.zeros(n, dtype=torch.float32, device=dev)
        self.views = []
        off = 0
        for p in self.params:
            k = p.numel()
            self.views.append(self.flat[off:off + k].view_as(p))
            off += k
        self.bind_()

    def bind_(self):
        """Point every .grad at its bucket view (copying a gradient some other code put there)."""
        for p, v in zip(self.params, self.views):
            g = p.grad
            if g is None or g.data_ptr() != v.data_ptr():
                if g is not None:
                    v.copy_(g)
                else:
                    v.zero_()
                p.grad = v

    def all_reduce_(self):
        if not active():
            return
        self.bind_()   # no-op unless a .grad was replaced
        timed = self.timing is not None and self.flat.is_cuda
        if timed:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        all_reduce_mean_(self.flat)
        if timed:
            ev[1].record()
            self.timing.append(ev)

    timing = None   # a list: every all_reduce_ appends its (start, stop) CUDA events (tools/bench_ppo.py)

    def all_reduce_ms(self):
        """Mean milliseconds of the timed all-reduces (synchronises)."""
        if not self.timing:
            return None
        torch.cuda.synchronize(self.flat.device)
        return sum(a.elapsed_time(b) for a, b in self.timing) / len(self.timing)

    def broadcast_params_(self, src=0):
        """Start every rank from rank src's weights."""
        if not active():
            return
        for p in self.params:
            x = p.data.to(_comm_device(p))
            dist.broadcast(x, src)
            if x is not p.data:
                with torch.no_grad():
                    p.copy_(x)   # through the parameter (not .data): its version counter moves, so packed weights follow
