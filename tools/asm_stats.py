#!/usr/bin/env python3
"""Static code statistics of the megakernel instantiations (no GPU needed).

Compiles bidirectional-pathtracing_amd/csrc/bdpt_hip.hip for gfx950 to assembly with the product
flags (plus any extra -D flags given on the command line) and prints, per k_bdpt_sample
instantiation: VGPRs, scratch bytes per lane, code size, instruction count, scratch / VMEM / LDS
instruction counts and exec-mask bookkeeping. Used to pre-screen A/B variants before a GPU run.

  python3 tools/asm_stats.py [-DFOO=1 ...]     (ASM_EXTRA="-mllvm ..." adds other compiler flags)
"""
import os
import re
import shlex
import subprocess
import sys
from collections import Counter

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CS = os.environ.get('ASM_CS', os.path.join(ROOT, 'bidirectional-pathtracing_amd', 'csrc'))
sys.path.insert(0, ROOT)
import __graft_entry__ as ge  # noqa: E402

extra = [a for a in sys.argv[1:] if a.startswith("-D")] + shlex.split(os.environ.get("ASM_EXTRA", ""))
tag = re.sub(r"[^A-Za-z0-9]+", "_", "_".join(extra)).strip("_")[:80] or "default"
out = f"/tmp/asm_{tag}.s"
cmd = [ge.HIPCC] + [f for f in ge.HIP_FLAGS if f not in ("-fPIC",)] + [
    "-I" + os.path.join(ROOT, "include"), "-I" + CS, "--cuda-device-only", "-S",
    os.path.join(CS, "bdpt_hip.hip"), "-o", out] + extra
subprocess.run(cmd, check=True, stderr=subprocess.DEVNULL)
s = open(out).read().split("\n")
want = re.compile(r"^(_ZN12_GLOBAL__N_113k_bdpt_sampleILi(\d+)ELb0ELi(\d)ELb(\d)EEEvNS_7KParamsE):")
for i, line in enumerate(s):
    m = want.match(line)
    if not m:
        continue
    name, maxv, lm, ext = m.groups()
    j = i
    while not s[j].startswith(".Lfunc_end"):
        j += 1
    body = s[i:j]
    tail = s[j:j + 40]
    info = {}
    for t in tail:
        mm = re.match(r"; (NumVgprs|ScratchSize|codeLenInByte|Occupancy)\s*[:=]\s*(\d+)", t.strip())
        if mm:
            info[mm.group(1)] = int(mm.group(2))
    ins = [l.split()[0] for l in body if l.startswith("\t") and not l.startswith("\t.") and l.split()
           and not l.strip().startswith(";")]
    c = Counter(ins)
    scr = sum(v for k, v in c.items() if k.startswith("scratch_"))
    vm = sum(v for k, v in c.items() if k.startswith("global_") or k.startswith("buffer_"))
    ds = sum(v for k, v in c.items() if k.startswith("ds_"))
    ex = sum(v for k, v in c.items() if "saveexec" in k or k.startswith("s_or_b64") or k.startswith("s_andn2_b64"))
    print(f"MAXV={maxv} LM={lm} EXT={ext}: vgpr {info.get('NumVgprs')} scratch {info.get('ScratchSize')} "
          f"code {info.get('codeLenInByte')} insts {len(ins)} scratch_ops {scr} vmem {vm} ds {ds} "
          f"exec_ops {ex} v_mov {c['v_mov_b32_e32']} cndmask {c['v_cndmask_b32_e32'] + c['v_cndmask_b32_e64']}")
