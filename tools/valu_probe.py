"""Run tools/valu_probe.hip: cycles per wave-instruction per SIMD for the VALU
instructions of the SHA-512 compression (K4's VALU roofline).

    python tools/valu_probe.py        (needs tools/_valu_probe.so, built in the container)
"""
import ctypes
import json
import os
import sys

import torch

HERE = os.path.dirname(os.path.abspath(__file__))
KINDS = ["v_lshl_add_u64", "v_add_co_u32+v_addc_co_u32 (64-bit add)", "v_alignbit_b32", "v_bitop3_b32",
         "v_xor_b32", "v_add_u32"]
CH = 8


def main():
    lib = ctypes.CDLL(os.path.join(HERE, "_valu_probe.so"))
    lib.valu_probe.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_void_p]
    dev = torch.device("cuda", 0)
    n_cu = torch.cuda.get_device_properties(0).multi_processor_count
    clk_ghz = float(sys.argv[1]) if len(sys.argv) > 1 else 2.4
    res = {}
    for waves_per_simd in (1, 2, 4, 8):
        blocks = n_cu * waves_per_simd  # 256-thread blocks = 4 waves = one per SIMD
        out = torch.empty(blocks * 256, dtype=torch.int64, device=dev)
        iters = 4000
        s = torch.cuda.current_stream().cuda_stream
        for kind in range(len(KINDS)):
            lib.valu_probe(kind, out.data_ptr(), blocks, 10, s)
            torch.cuda.synchronize()
            ts = []
            for _ in range(3):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                lib.valu_probe(kind, out.data_ptr(), blocks, iters, s)
                e1.record()
                torch.cuda.synchronize()
                ts.append(e0.elapsed_time(e1) * 1e-3)
            t = min(ts)
            instr_per_simd = waves_per_simd * iters * CH  # wave-instructions each SIMD issued
            if kind == 1:
                instr_per_simd *= 2  # two instructions per 64-bit add
            cyc = t * clk_ghz * 1e9 / instr_per_simd
            res.setdefault(KINDS[kind], {})[f"{waves_per_simd}w"] = round(cyc, 3)
    print(json.dumps({"cycles_per_wave_instr_per_simd_at_%.1fGHz" % clk_ghz: res}, indent=1))


if __name__ == "__main__":
    main()
