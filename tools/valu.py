"""VALU-side roofline record of the env kernel from the rocprofv3 SQ passes
(tools/pmc_sq.sh -> tools/pmc_summary.py output) -> profiles/valu.json,
keyed like bench.py's lookup '<env_id>/fp<precision>/<envs>'.

Per launch (counters averaged over the step dispatches):
  fp64 flop      = 64 lanes x lane activity x (2 FMA + MUL + ADD) wave-instructions,
                   lane activity = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU);
  achieved       = fp64 flop / kernel time, against the 78.6 TFLOP/s fp64 vector peak
                   (256 CU x 4 SIMD x 16 fp64 FMA lanes/clk x 2 x 2.4 GHz);
  valu_active    = SQ_ACTIVE_INST_VALU / SQ_WAVE_CYCLES (share of wave time issuing VALU);
  lds conflicts  = SQ_LDS_BANK_CONFLICT against SQ_ACTIVE_INST_LDS.

    python tools/valu.py <pmc_summary.txt> <kernel_ms> <env_id> <precision> <envs> <source>
"""
import json
import os
import re
import sys

PEAK_TF = 78.6


def read_summary(path):
    vals = {}
    for line in open(path):
        m = re.match(r'(\S+)\s+([-+0-9.eE]+)', line)
        if m:
            vals[m.group(1)] = float(m.group(2))
    return vals


def record(v, kernel_ms, source):
    inst = 2 * v['SQ_INSTS_VALU_FMA_F64'] + v['SQ_INSTS_VALU_MUL_F64'] + v['SQ_INSTS_VALU_ADD_F64']
    lanes = v['SQ_THREAD_CYCLES_VALU'] / (64.0 * v['SQ_ACTIVE_INST_VALU'])
    flop = 64.0 * lanes * inst
    tf = flop / (kernel_ms * 1e-3) / 1e12
    return {'bound': 'valu-latency', 'fp64_tflops': tf, 'peak_tflops': PEAK_TF, 'frac': tf / PEAK_TF,
            'fp64_flop_per_launch': flop, 'lane_activity': lanes,
            'valu_insts_per_launch': v['SQ_INSTS_VALU'],
            'valu_active_frac': v['SQ_ACTIVE_INST_VALU'] / v['SQ_WAVE_CYCLES'],
            'lds_bank_conflict_cycles': v['SQ_LDS_BANK_CONFLICT'], 'lds_active_cycles': v['SQ_ACTIVE_INST_LDS'],
            'lds_conflict_over_active': v['SQ_LDS_BANK_CONFLICT'] / v['SQ_ACTIVE_INST_LDS'],
            'kernel_ms': kernel_ms, 'source': source}


def issue_analysis(v, kernel_ms, waves=1024, clock_ghz=2.4):
    """VALU issue against its ceiling and where the other wave cycles go.
    One wave alone on its SIMD issues a VALU instruction per 4 cycles (8 for
    a transcendental; MI355X_MICROARCH.md constants, 'vector-instruction
    ISSUE cost'), so the kernel's issue floor is its VALU instructions per
    wave x 4 cycles; the SQ shares are fractions of SQ_WAVE_CYCLES:
    ACTIVE_INST_ANY (some instruction issuing), WAIT_INST_ANY (at an
    s_waitcnt: LDS / memory), and the residual — cycles with no instruction
    issued and no waitcnt — which is the dependent-instruction latency of
    the wave's own VALU chain (no SQ counter of its own)."""
    per_wave = (v['SQ_INSTS_VALU'] + v.get('SQ_INSTS_VALU_TRANS_F64', 0) + v.get('SQ_INSTS_VALU_TRANS_F32', 0)) / waves
    floor_cycles = 4.0 * per_wave
    kernel_cycles = kernel_ms * 1e-3 * clock_ghz * 1e9
    w = v['SQ_WAVE_CYCLES']
    return {'valu_issue_floor_us': floor_cycles / (clock_ghz * 1e3), 'issue_ceiling_frac': floor_cycles / kernel_cycles,
            'wave_cycle_shares': {'valu_issuing': v['SQ_ACTIVE_INST_VALU'] / w, 'any_issuing': v['SQ_ACTIVE_INST_ANY'] / w,
                                  'waitcnt': v['SQ_WAIT_INST_ANY'] / w, 'waitcnt_lds': v['SQ_WAIT_INST_LDS'] / w,
                                  'dependency_residual': 1.0 - (v['SQ_ACTIVE_INST_ANY'] + v['SQ_WAIT_INST_ANY']) / w},
            'waves': waves, 'clock_ghz': clock_ghz}


def main():
    summ, kms, env_id, prec, n, source = sys.argv[1:7]
    rec = record(read_summary(summ), float(kms), source)
    out = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), 'profiles', 'valu.json')
    db = json.load(open(out)) if os.path.exists(out) else {}
    db[f'{env_id}/fp{prec}/{n}'] = rec
    json.dump(db, open(out, 'w'), indent=1, sort_keys=True)
    print(json.dumps(rec))


if __name__ == '__main__':
    main()
