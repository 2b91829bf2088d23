"""Processor cases shared by make_golden_processor.py (fixture generation) and
tests/test_processor_cpu.py: conversations x mode, built with the processor's own message helpers."""
import numpy as np
import torch


def codes(seed, T, n_vq=4):
    return torch.from_numpy(np.random.default_rng(seed).integers(0, 1024, (T, n_vq)))


def cases(P):
    u = P.build_user_message
    a = P.build_assistant_message
    return {
        "gen_text": ([[u(text="Hello world.")]], "generation"),
        "gen_clone": ([[u(text="Say this.", reference=[codes(1, 7)])]], "generation"),
        "gen_fields": ([[u(text="Calm voice.", instruction="calm", language="en", tokens=12, quality="high")]],
                       "generation"),
        "gen_batch": ([[u(text="Short.")], [u(text="A longer sentence here.", reference=[codes(2, 5)])]], "generation"),
        "gen_multiturn": ([[u(text="First."), a([codes(3, 6)]), u(text="Second.")]], "generation"),
        "cont": ([[u(text="Go on."), a([codes(4, 5)])]], "continuation"),
    }
