"""GPU: the opt-in / A-B paths that the default run does not take, each held to the fp64 oracle in
a subprocess (the library reads its switches once per process):

  DSTAGNN_DE_OMAP=1    the inner block's dE accumulated into dx by the GEMM output-map epilogue
                       (block.hip stage_tat) instead of a dE buffer + transpose_kernel
  DSTAGNN_TAT_MFMA=0   the VALU wave kernels of the temporal attention instead of the
                       matrix-core ones (ops.hip tat_*_mfma_kernel)
  DSTAGNN_SIDE_CUMASK  the side stream confined to a CU subset (scheduling only: same results)
  DSTAGNN_SDDMM_NOPF=1 the aggregate-first SDDMM without its batch prefetch (4 waves per SIMD)
  DSTAGNN_SDDMM_PAIR=0 the aggregate-first SDDMM one sample per wave instead of sample pairs
                       (=1 with B = 3: the default pair kernel with an odd batch, a lone last sample)
  DSTAGNN_AGG_PAIR=0   the aggregate-first forward and transposed SpMM one sample per wave instead
                       of sample pairs (=1 with B = 3: the pair kernels with a lone last sample)
  DSTAGNN_FLASH_DQK2=0 the small-graph dQ' / dK' kernel one strip per workgroup instead of two
                       (N <= 192)
  DSTAGNN_FLASH_MASK2=0 the small-graph mask gradient summing the batch per thread instead of
                       over a wave's lanes
  DSTAGNN_TF_WAVES=4 / DSTAGNN_TF_BWD_WAVES=4  the fused temporal-attention kernels on four waves
                       instead of eight
  DSTAGNN_GTU_TCONV=0  the GTU input gradient as the K-concatenated GEMM (run_gemm_kcat)
  DSTAGNN_GTU_GCONV=1  the GTU forward convolutions by the sliding-window kernel (gtu_tconv.hip)
  DSTAGNN_TAIL_CT24=0  the split GTU tail path at T = 24 instead of the compile-time kernels
  DSTAGNN_KSIG=0       main -> side stream forks signalled by hipStreamWriteValue32 instead of
                       by the next main-stream kernel's prologue store (block.hip Streams::fork;
                       the default path is held by every other GPU test)
  DSTAGNN_FC_SIDE=1    the TAt fc weight gradient on the side stream instead of grouped with the
                       Q|K|V weight gradient on the main stream
  DSTAGNN_TATLN_SIDE=1 the TAt LayerNorm gamma / beta column sums on the side stream
  DSTAGNN_GATES_BWD_SCALAR=1  the split-path GTU gates backward one element per thread (T = 144)
  DSTAGNN_TAT_FUSED=0  the temporal-attention stage as separate launches (Q|K|V GEMM, attention,
                       fc GEMM, LayerNorm, x transpose) instead of tat_fused.hip's one kernel
  DSTAGNN_TAIL_FOLD=1  the GTU tail backward folds its LayerNorm / residual_conv partial sums
                       in-kernel (ticket tree over grid-stride workgroups) instead of colsum2d
  DSTAGNN_GTU_FUSED=0  the GTU stage forward as the grouped conv GEMM + gtu_tail_fwd_ct instead of
                       gtu_fused.hip's one kernel (convolutions, gates, fcmy, residual, LN)
  DSTAGNN_GTU_FUSED_BWD=0  the GTU stage backward as gtu_tail_bwd_ct + gtu_tconv (zero-padded gate
                       gradient rows) instead of gtu_fused.hip's one kernel
  DSTAGNN_SATLN_FUSED=1  the SAt projection backward (dZd GEMM) and the EmbedS LayerNorm backward as one
                       kernel (sat_fused.hip) instead of a GEMM + ln_bwd
  DSTAGNN_LN_V4=0      the LayerNorm rows of 256 / 512 / 1024 floats by the scalar wave-per-row kernels
                       instead of the float4 ones
  DSTAGNN_DWP_MAIN=1   the pre_conv weight gradient on the main stream instead of the side stream
  DSTAGNN_DEBUG_STREAMS=1  the fork invariant asserted (block.hip Bwd::sq): no side-stream work
                       issued while a fork's signal is still pending
  DSTAGNN_DEBUG_MAIN_DELAY_US / DSTAGNN_DEBUG_SIDE_DELAY_US   race probes: a 1.5 ms busy-wait
                       kernel on the main stream before every stage / on the side stream after
                       every fork, so a cross-stream read without its dependency reads stale
                       data (block.hip debug_delay); results must not change

PEMS08 geometry (the bench's default path otherwise; t24 for the T = 24 switches), inner block
with a broadcast res_att in eval and train mode plus the first block, same bounds as
tests/test_gpu_parity.py::test_block_vs_oracle_configs."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

pytestmark = pytest.mark.gpu

SCRIPT = """
import sys
sys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})
import test_gpu_parity as T
T._run_config_vs_oracle({cfg!r}, False, {B}, flash={flash!r})
T._run_config_vs_oracle({cfg!r}, False, {B}, train=True, flash={flash!r})
T._run_config_vs_oracle({cfg!r}, True, 2, flash={flash!r})
print("KNOB_OK")
"""


@pytest.mark.parametrize("env,cfg,B", [("DSTAGNN_DE_OMAP=1", "pems08", 4), ("DSTAGNN_TAT_MFMA=0", "pems08", 4),
                                       ("DSTAGNN_SIDE_CUMASK=0x11111111", "pems08", 4),
                                       ("DSTAGNN_SDDMM_NOPF=1", "pems08", 4), ("DSTAGNN_GTU_TCONV=0", "pems08", 4),
                                       ("DSTAGNN_SDDMM_PAIR=0", "pems08", 4), ("DSTAGNN_SDDMM_PAIR=1", "pems08", 3),
                                       ("DSTAGNN_AGG_PAIR=0", "pems08", 4), ("DSTAGNN_AGG_PAIR=1", "pems08", 3),
                                       ("DSTAGNN_FLASH_DQK2=0", "pems08", 4), ("DSTAGNN_FLASH_MASK2=0", "pems08", 4),
                                       ("DSTAGNN_TF_WAVES=4", "pems08", 4), ("DSTAGNN_TF_BWD_WAVES=4", "pems08", 4),
                                       ("DSTAGNN_GTU_GCONV=1", "pems08", 4), ("DSTAGNN_GTU_GCONV=1", "t24", 2),
                                       ("DSTAGNN_TAIL_CT24=0", "t24", 2), ("DSTAGNN_KSIG=0", "pems08", 4),
                                       ("DSTAGNN_KSIG=0", "pems07+flash", 2), ("DSTAGNN_FC_SIDE=1", "pems08", 4),
                                       ("DSTAGNN_TATLN_SIDE=1", "pems08", 4),
                                       ("DSTAGNN_DEBUG_MAIN_DELAY_US=1500", "pems08", 4),
                                       ("DSTAGNN_DEBUG_SIDE_DELAY_US=1500", "pems08", 4),
                                       ("DSTAGNN_DEBUG_MAIN_DELAY_US=1500", "pems07+flash", 2),
                                       ("DSTAGNN_GATES_BWD_SCALAR=1", "t144k3", 2),
                                       ("DSTAGNN_DEBUG_STREAMS=1", "pems08", 4),
                                       ("DSTAGNN_TAT_FUSED=0", "pems08", 4),
                                       ("DSTAGNN_TAIL_FOLD=1", "pems08", 4),
                                       ("DSTAGNN_GTU_FUSED=0", "pems08", 4), ("DSTAGNN_GTU_FUSED_BWD=0", "pems08", 4),
                                       ("DSTAGNN_SATLN_FUSED=1", "pems08", 4), ("DSTAGNN_LN_V4=0", "pems08", 4),
                                       ("DSTAGNN_DWP_MAIN=1", "pems08", 4),
                                       ("DSTAGNN_DEBUG_STREAMS=1", "pems07+flash", 2)])
def test_knob_path_vs_oracle(env, cfg, B):
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    k, v = env.split("=", 1)
    e = dict(os.environ, PYTHONDONTWRITEBYTECODE="1")
    e[k] = v
    flash = True if cfg.endswith("+flash") else None  # "+flash": the streamed (large-graph) kernels forced on
    cfg = cfg.split("+")[0]
    code = SCRIPT.format(root=ROOT, tests=os.path.join(ROOT, "tests"), cfg=cfg, B=B, flash=flash)
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=e, capture_output=True, text=True, timeout=170)
    assert r.returncode == 0 and "KNOB_OK" in r.stdout, (r.stdout[-2000:], r.stderr[-3000:])


def test_race_probe_catches_a_missing_fork():
    """The main-stream delay probe against a library built with one cross-stream dependency
    removed on purpose (the TAt LayerNorm column sums issued on the side stream without a
    fork: block.hip under -DDSTAGNN_RACEBUG_NOFORK, built by `make` into abtest/racebug from the
    same sources as the shipped library): the parity check must FAIL there, i.e. the probe
    exposes a missing fork instead of hiding it.  DSTAGNN_POISON=1: the racing read sees NaN
    scratch, not a previous run's equal values."""
    import torch
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    lib = os.path.join(ROOT, "abtest", "racebug", "libdstagnn.so")
    assert os.path.exists(lib), "abtest/racebug/libdstagnn.so missing: run `make` (target racebug)"
    e = dict(os.environ, PYTHONDONTWRITEBYTECODE="1", DSTAGNN_DEBUG_MAIN_DELAY_US="3000", DSTAGNN_POISON="1",
             LD_LIBRARY_PATH=os.path.dirname(lib))
    code = ("import sys\nsys.path.insert(0, {root!r}); sys.path.insert(0, {tests!r})\n"
            "import test_gpu_parity as T\n"
            "T._run_config_vs_oracle('pems08', False, 4, train=True)\nprint('KNOB_OK')\n"
            ).format(root=ROOT, tests=os.path.join(ROOT, "tests"))
    r = subprocess.run([sys.executable, "-c", code], cwd=ROOT, env=e, capture_output=True, text=True, timeout=170)
    assert "KNOB_OK" not in r.stdout and "AssertionError" in r.stderr, (r.stdout[-1500:], r.stderr[-1500:])
