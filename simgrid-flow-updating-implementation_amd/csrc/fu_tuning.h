// fu_tuning.h — the engine's compile-time tuning constants, in one place.
//
// Each value below is the shipped one, with the measurement that chose it. None of them is a
// build switch any more: the experiment builds of rounds 2-5 (`make VARIANT=... EXTRA=-D...`)
// are gone, so the kernels compile one way only. Changing a value here is a code change that
// the GPU parity suite must re-verify (the arithmetic is unchanged by every one of them; they
// move work between lanes, launches and caches only).
#ifndef FU_TUNING_H_
#define FU_TUNING_H_

// Exact fp64 chains (heavy rows, mega hubs): elements per LDS batch of the lane-uniform chain.
// One wave alone: 8 -> 8.75, 16 -> 7.2, 32 -> 6.4 ns per element; 32 costs registers the heavy
// launches need for occupancy. The register launch of kernel 9 uses
// 8-element batches to stay at 166 VGPRs (§4.12).
constexpr int kChainB = 16;

// k_stage: steps per lane whose column loads are in flight per batch (doubles: 16 B per step).
// 2 / 4 / 8 gave 61.9 / 63.1 / 63.8 us per ER-1M round in one screen and 63.0 / 63.0 in four
// more pairs; the 1000-round job alike (profiles/r05/ab, ac). 4 kept.
constexpr int kStageU = 4;

// k_stage stores its staged doubles non-temporal (G is streamed out once and read back by the
// next launch): ER-1M 61.8 vs 62.7 us, R-MAT-24 6,728 vs 6,807 us per round (profiles/r05/n, o).
// The packed codes (1-4 byte elements, 8-32 MB) stay write-back: they fit on chip until the
// tiles read them (non-temporal there: 41.0 vs 38.8 us per 8-bit round, profiles/r05/q, r).
constexpr int kStageNtMinBytes = 8;

// k_transpose: minimum blocks per CU in its launch bounds (one 1024-thread block per CU,
// persistent over its XCD's buckets; 2 per CU spilled 36 B and measured within the spread).
constexpr int kTrWaves = 1;

// Persistent tick replay: s_sleep units (64 cycles each) a wave waits after a pass over its
// lanes that made no progress (profiles/r03/pairwise: longer sleeps did not change the tick).
constexpr int kReplaySleep = 2;

// Kernel 8 light tiles: edges x rows per tile. 512 x 64 ran 67.3-72.5 against 57.8-62.5 us
// per ER-1M round (profiles/r05/f); 1024 x 256 does not fit the u16 position|run index.
constexpr int kStageTE = 1024, kStageTN = 128;

// Kernel 9: directed edges per transpose bucket (one 1024-thread block; u16 positions).
// 16K-edge buckets +0.2 ms, 4K +0.4 ms per R-MAT-24 round.
constexpr int kTrBE = 8192;

// Kernel 4 heavy rows of up to 64 x kHeavyRL edges keep their operands in registers and write
// their flows from them; longer rows make a second pass (R-MAT-24: 9.35 -> 8.89 ms, round 2).
// 512 or 1024 elements per wave lost more in occupancy than the second pass costs (+0 %, +21 %).
constexpr int kHeavyRL = 4;

#endif  // FU_TUNING_H_
