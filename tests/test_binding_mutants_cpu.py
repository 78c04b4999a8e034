"""tools/binding_mutants.sh stays meaningful: every mutant's sed pattern
still matches a line of the shipped binding (integration/multiscale.array.
gpu.cpp), so each mutant really is the binding with one deliberate bug
(the GPU run of the mutants is recorded in profiles/r06_binding_mutants.
jsonl: every one fails tests/test_gpu_binding_exec.py)."""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_every_mutant_pattern_matches_the_binding():
    script = open(os.path.join(REPO, "tools", "binding_mutants.sh")).read()
    binding = open(os.path.join(REPO, "integration", "multiscale.array.gpu.cpp")).read()
    muts = re.findall(r"\[(\w+)\]='s/(.*?)/(.*?)/'", script)
    assert len(muts) == 6, muts
    for name, pat, rep in muts:
        # the patterns are literal text (sed's '.' matches itself too)
        assert pat in binding, f"mutant {name}: pattern no longer in the binding"
        assert pat != rep, name
