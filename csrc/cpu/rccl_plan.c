/*
 * rccl_plan.c -- the round plan of the single-process RCCL job
 * (otc_multi_run strategy 1, csrc/hip/pipeline.cpp rccl_job_run) as a pure
 * function, so the N = 2..8 plan (round offsets, per-GPU pieces, CTR block
 * offsets, CBC-decryption halo slots, last-round padding) is unit-tested on
 * the CPU (tests/test_rccl_plan_cpu.py) against the Python planner
 * (our_tree_amd/parallel/shard.py) and the oracle -- RCCL refuses two ranks
 * on one GPU, so the GPU path itself only ever runs with ngpus = 1 here.
 *
 * The reference chunks a buffer per pthread and drops the remainder
 * (/root/reference/test.c:44-58, 94-112); this plan covers every byte: a
 * piece past the end is empty and the last round's root buffer is zero-padded
 * to the equal counts ncclScatter / ncclGather need.
 */
#include "otc.h"

uint64_t otc_rccl_nrounds(uint64_t nbytes, int ngpus, uint64_t piece)
{
    if (ngpus < 1 || piece == 0) return 0;
    const uint64_t round = piece * (uint64_t)ngpus;
    return (nbytes + round - 1) / round;
}

uint64_t otc_rccl_halo_start(uint64_t nbytes, uint64_t piece, uint64_t i)
{
    const uint64_t s = i * piece;
    return s < nbytes ? s : nbytes;
}

int otc_rccl_plan_piece(uint64_t nbytes, int ngpus, uint64_t piece, uint64_t r, int g, otc_rccl_piece *out)
{
    if (!out || ngpus < 1 || piece == 0 || g < 0 || g >= ngpus) return OTC_ERR_ARG;
    const uint64_t nr = otc_rccl_nrounds(nbytes, ngpus, piece);
    if (r >= nr) return OTC_ERR_ARG;
    const uint64_t round = piece * (uint64_t)ngpus;
    out->round_off = r * round;
    out->round_bytes = nbytes - out->round_off < round ? nbytes - out->round_off : round;
    out->pad_bytes = round - out->round_bytes;
    out->off = out->round_off + (uint64_t)g * piece;
    out->bytes = out->off < nbytes ? (nbytes - out->off < piece ? nbytes - out->off : piece) : 0;
    if (out->off > nbytes) out->off = nbytes; /* an empty piece past the end */
    out->blk0 = out->off / 16;
    /* the halo slot of piece (r, g) is r * ngpus + g: its start is exactly off */
    out->halo = (out->bytes && out->off > 0) ? (int64_t)(r * (uint64_t)ngpus + (uint64_t)g) : -1;
    return OTC_OK;
}
