"""Row-group sharding across GPUs.

Row groups are independent units of the read path (FileReader.readRowGroupData
chunk_reader.go:375-404; dictionaries are per chunk, :196-228), so a file is
partitioned by contiguous row-group ranges, one range per rank, each decoded
on its own GPU with its own streams. There is no collective on the data path;
the only cross-rank operation is the max-over-ranks of the step time the
benchmark reports.
"""


def row_group_range(num_row_groups, rank, world):
    """[first, last) row groups of `rank` out of `world`: contiguous, disjoint, covering."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError(f"bad rank {rank} of {world}")
    return num_row_groups * rank // world, num_row_groups * (rank + 1) // world


def max_over_ranks(value, dist=None, device="cpu"):
    """max(value) over the ranks of the default process group (value itself without one)."""
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return float(value)
    import torch
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def gather_column(local, dist=None):
    """The whole column on every rank from each rank's decoded slice (the
    optional collective): rank r contributes its row-group range's values, in order, and every
    rank receives the concatenation in rank order. One all-gather of the slice sizes, then one
    all_gather_into_tensor of the slices padded to the largest (RCCL over xGMI on GPUs, gloo on
    CPU). Not on the decode path: the benchmark times it separately (`bench.py --gather`)."""
    import torch
    if dist is None or not dist.is_initialized() or dist.get_world_size() == 1:
        return local
    world = dist.get_world_size()
    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    sizes = torch.empty(world, dtype=torch.int64, device=local.device)
    dist.all_gather_into_tensor(sizes, n)
    sizes = [int(s) for s in sizes.cpu()]
    m = max(sizes)
    buf = local if local.numel() == m else torch.cat([local, local.new_zeros(m - local.numel())])
    out = local.new_empty(world * m)
    dist.all_gather_into_tensor(out, buf.contiguous())
    if all(s == m for s in sizes):
        return out
    return torch.cat([out[r * m: r * m + s] for r, s in enumerate(sizes)])


def device_values(batch, chunk_ids, device):
    """This rank's decoded values of `chunk_ids` (fixed-width columns) concatenated into one
    torch tensor on `device`, copied device to device from the batch's output arena (no host
    round trip). The element type is the column's 8-byte lane (int64 view) or int32.
    The copies go through pqgpu_copy, i.e. the HIP runtime libpqgpu itself is bound to. torch must
    initialise HIP before libpqgpu is loaded (bench.py does): torch ships its own libamdhip64
    (soname libamdhip64.so.7), which libpqgpu then binds to, so the process has one HIP runtime
    and the two share device pointers."""
    import torch
    from . import copy as pq_copy
    rs = [batch.result(c, copy=False) for c in chunk_ids]
    width = {r.value_width for r in rs}
    if len(width) != 1 or width.pop() not in (4, 8):
        raise ValueError("device_values: one fixed width of 4 or 8 bytes expected")
    dt = torch.int64 if rs[0].value_width == 8 else torch.int32
    out = torch.empty(sum(r.num_values for r in rs), dtype=dt, device=device)
    torch.cuda.synchronize(device)
    at = 0
    for r in rs:
        nb = r.num_values * r.value_width
        if nb:
            pq_copy(batch_ctx(batch), out.data_ptr() + at, r.values, nb)
        at += nb
    return out


def batch_ctx(batch):
    if batch.ctx is None:
        raise ValueError("device_values needs a batch with a device context")
    return batch.ctx
