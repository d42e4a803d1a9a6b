"""Static issue-cost summary of kernels in a gfx950 assembly file (hipcc --cuda-device-only -S).

    python tools/isa_cost.py win.s window_features_reg_kernelILi3ELi8ELb1 [...]

Per matching kernel: VALU / SALU / LDS / VMEM instruction counts, a weighted VALU cost in wave64
issue units of 2 cycles (packed f32 and 64-bit shifts 2 units — their lane rate is half the scalar
f32 rate on the 32-wide SIMD — transcendentals 4), VGPRs and scratch.  A counting aid for A/B of
kernel variants before a GPU run, not a timing model."""
import re
import sys

WEIGHT = [(re.compile(r"v_pk_(fma|add|mul)_f32"), 2), (re.compile(r"v_(lshlrev|lshrrev|ashrrev)_[bi]64|v_lshl_add_u64"), 2),
          (re.compile(r"v_(sqrt|rsq|rcp|exp|log|sin|cos)_f32"), 4)]


def kernels(path):
    txt = open(path).read().split("\n")
    i = 0
    while i < len(txt):
        m = re.match(r"^(_Z\S+):", txt[i])
        if not m:
            i += 1
            continue
        j = i + 1
        while j < len(txt) and not txt[j].startswith(".Lfunc_end"):
            j += 1
        meta = "\n".join(txt[j:j + 400])
        yield m.group(1), txt[i:j], meta
        i = j


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    for name, body, meta in kernels(path):
        if pats and not any(p in name for p in pats):
            continue
        ops = [ln.split()[0] for ln in body if re.match(r"\s+[a-z]", ln) and not ln.strip().startswith(";")]
        valu = [o for o in ops if o.startswith("v_")]
        cost = 0
        for o in valu:
            w = 1
            for rx, ww in WEIGHT:
                if rx.match(o):
                    w = ww
            cost += w
        vg = re.search(r"NumVgprs: (\d+)", meta)
        sc = re.search(r"ScratchSize: (\d+)", meta)
        print(f"{name[:110]}\n   VALU {len(valu)} (cost {cost})  SALU {sum(o.startswith('s_') for o in ops)}  "
              f"LDS {sum(o.startswith('ds_') for o in ops)}  VMEM {sum(o.startswith(('global_', 'buffer_')) for o in ops)}  "
              f"vgpr {vg and vg.group(1)}  scratch {sc and sc.group(1)}")


if __name__ == "__main__":
    main()
