"""Data-parallel generate across GPUs: one process per GPU, each owning a full engine
replica; a batch of utterances is split into contiguous row shards.

There is no collective inside the decode loop.  The only exchange is the gather of the
finished rows (a few KB of token ids per utterance), after which every row is right-padded
to the global step count with [pad_token_id, audio_pad x n_vq] rows -- exactly the rows
the reference appends to a stopped sequence while the rest of its batch is still running
(`moss_tts_delay/modeling_moss_tts.py:453,475,513`) -- so the gathered result equals a
single-process generate() over the whole batch.

Shards keep the GLOBAL left padding (rows are sliced from the globally padded tensors),
because positions include pads (`TF/.../modeling_qwen3.py:386-389`).  With
audio_repetition_penalty != 1 the reference couples rows through a batch-wide penalty set
(`inference_utils.py:79-88`); sharding then changes results, as documented in DESIGN.md.
"""
from typing import Callable, List, Optional, Tuple

import torch


def shard_bounds(n_rows: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous split; shard sizes differ by at most one (earlier ranks take the extra)."""
    base, extra = divmod(n_rows, world)
    start = rank * base + min(rank, extra)
    return start, start + base + (1 if rank < extra else 0)


def _dist():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


def pad_to_steps(outputs: List[Tuple[int, torch.Tensor]], prompt_len: int, pad_token_id: int,
                 audio_pad_code: int) -> List[Tuple[int, torch.Tensor]]:
    """Right-pad every row to the largest number of generated steps in the list."""
    # ids = generation_ids[start:] = (prompt_len - start) prompt rows + n_steps rows, and
    # start_length = prompt_len - start, so n_steps = len(ids) - start_length
    steps = [int(ids.shape[0]) - int(sl) for sl, ids in outputs]
    n = max(steps) if steps else 0
    out = []
    for (sl, ids), k in zip(outputs, steps):
        if k < n:
            pad = torch.full((n - k, ids.shape[1]), audio_pad_code, dtype=ids.dtype, device=ids.device)
            pad[:, 0] = pad_token_id
            ids = torch.cat([ids, pad], 0)
        out.append((sl, ids))
    return out


def generate_dp(generate_fn: Callable, input_ids: torch.Tensor, attention_mask: Optional[torch.Tensor],
                pad_token_id: int = 151643, audio_pad_code: int = 1024, **kwargs):
    """Run `generate_fn(input_ids_shard, attention_mask_shard, **kwargs)` (the model's
    generate()) on this rank's rows and return the full batch's outputs on every rank."""
    dist, rank, world = _dist()
    B, T = int(input_ids.shape[0]), int(input_ids.shape[1])
    s, e = shard_bounds(B, world, rank)
    local = []
    if e > s:
        am = attention_mask[s:e] if attention_mask is not None else None
        local = [(int(sl), ids.detach().cpu()) for sl, ids in generate_fn(input_ids[s:e], am, **kwargs)]
    if world == 1:
        gathered = [local]
    else:
        gathered = [None] * world
        dist.all_gather_object(gathered, local)
    flat = [row for part in gathered for row in part]
    return pad_to_steps(flat, T, pad_token_id, audio_pad_code)
