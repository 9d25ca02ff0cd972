"""Static checks of the built gfx950 code (no GPU): the hand-written DPP multiply-adds
(step.hip fmac_rowb / fmac3_rowb, inline asm) must not be followed directly by a DPP instruction
that reads one of the registers they wrote -- the compiler's hazard recognizer does not see inline
asm as a VALU definition, and a VALU write followed by a DPP read of the same VGPR needs two wait
states.  The asm blocks start with their own s_nop for the hazard on their inputs."""
import re
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def _disasm():
    # blocked mode (the sparse PGS) and the 16-lane kernels (the dense register PGS)
    objs = sorted(o for o in (ROOT / "build" / "obj").glob("hip_step.hip.part*.o") if o.name != "hip_step.hip.part0.o")
    if not objs:
        pytest.skip("no step.hip objects in build/obj (library built elsewhere)")
    r = subprocess.run(["bash", str(ROOT / "scripts" / "disasm.sh"), *map(str, objs)], capture_output=True, text=True,
                       check=True)
    return r.stdout.split("\n")


def test_no_dpp_read_after_asm_fmac():
    lines = _disasm()
    n_asm, bad = 0, []
    i = 0
    while i < len(lines):
        if "v_fmac_f32_dpp" not in lines[i]:
            i += 1
            continue
        dsts = set()
        j = i
        while j < len(lines) and "v_fmac_f32_dpp" in lines[j]:
            dsts.add(re.search(r"v_fmac_f32_dpp (v\d+)", lines[j]).group(1))
            j += 1
        n_asm += 1
        for t in range(j, min(j + 2, len(lines))):
            ins = lines[t].split("//")[0]
            if "s_nop" in ins:
                break
            if any(k in ins for k in ("row_", "quad_perm", "_dpp")):
                regs = re.findall(r"\bv\d+\b", ins)
                if len(regs) > 1 and regs[1] in dsts:
                    bad.append("\n".join(lines[i:t + 1]))
        i = j
    assert n_asm > 0
    assert not bad, bad[:3]
