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
