"""Exit protocol of the persistent traversal's work counters (CPU restatement).

The last wave of every persistent launch resets the dequeue heads for the next
launch (pupiloptixlab_amd/csrc/pt_kernels.hip, end of trace4_body): waves
count out on kWorkShards sub-counters (blockIdx % kWorkShards), the last wave
of each sub-counter on the final counter, and the last of those resets.  This
checks, for every grid size the launcher can produce and random exit orders,
that exactly one wave resets and that it is the last wave to leave.
"""
import os
import random
import re

HERE = os.path.dirname(os.path.abspath(__file__))
HDR = os.path.join(HERE, "..", "pupiloptixlab_amd", "csrc", "pt_kernels.h")


def constants():
    src = open(HDR).read()
    shards = int(re.search(r"kWorkShards = (\d+)", src).group(1))
    stride = int(re.search(r"kWorkStride = (\d+)", src).group(1))
    block = int(re.search(r"kTraceBlock = (\d+)", src).group(1))
    assert "kWorkKind = (2 * kWorkShards + 1) * kWorkStride" in src
    return shards, stride, block


def simulate(grid, shards, waves_per_block, rng):
    sub_cnt = [0] * shards
    final = 0
    waves = [(b, w) for b in range(grid) for w in range(waves_per_block)]
    rng.shuffle(waves)
    resets = []
    groups = min(grid, shards)
    for order, (b, _) in enumerate(waves):
        sub = b % shards
        sub_waves = (grid - sub + shards - 1) // shards * waves_per_block
        old = sub_cnt[sub]
        sub_cnt[sub] += 1
        if old == sub_waves - 1:
            old_f = final
            final += 1
            if old_f == groups - 1:
                resets.append(order)
    return resets, len(waves)


def test_exactly_the_last_wave_resets():
    shards, _, block = constants()
    wpb = block // 64
    rng = random.Random(7)
    for grid in list(range(1, 40)) + [255, 256, 257, 3583, 3584, 4096]:
        for _ in range(3):
            resets, n = simulate(grid, shards, wpb, rng)
            assert resets == [n - 1], (grid, resets, n)


def test_counter_layout_fits_the_allocation():
    shards, stride, _ = constants()
    kind = (2 * shards + 1) * stride
    # heads [0, shards), final exit counter at shards, sub-counters after it
    slots = [k * stride for k in range(2 * shards + 1)]
    assert max(slots) < kind and len(set(slots)) == len(slots)
