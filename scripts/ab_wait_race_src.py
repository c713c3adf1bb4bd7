"""Write build/abx/nuts_waitrace.hip: nuts.hip with the round-5 WAIT resolution restored (every
lane of a chain reads the transition count itself, as before the fix), for
scripts/diag_wait_race.py (experiment only; never shipped)."""
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = open(os.path.join(ROOT, "numpyro_amd", "csrc", "nuts.hip")).read()
rep = [
    ("  begin_step(cfg, a, c, valid, S, A, TPC == 1);\n", "  begin_step(cfg, a, c, valid, S, A, true);\n"),
    ("    if (vw == 0 && valid && S.phase == NMX_PH_WAIT) wait_go[cl] =", "    if (false) wait_go[cl] ="),
    ("    if (valid && S.phase == NMX_PH_WAIT && wait_go[cl]) begin_act(", "    if (false) begin_act("),
]
for a, b in rep:
    assert a in src, a[:70]
    src = src.replace(a, b, 1)
os.makedirs(os.path.join(ROOT, "build", "abx"), exist_ok=True)
open(os.path.join(ROOT, "build", "abx", "nuts_waitrace.hip"), "w").write(src)
