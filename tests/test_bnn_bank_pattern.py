"""k_bnn_c3's LDS layout claims (potential_bnn.hip, DESIGN.md 'BNN: register-blocked products'):
the k-lane permutation covers K exactly once, every operand read of the first 64 k of each of the
three products is bank-conflict-free, and the remainder steps are at most 2-way."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "scripts"))
import bnn_bank_pattern as BP  # noqa: E402


def test_bnn_c3_operand_reads_are_conflict_free():
    for name, (bijective, steps) in BP.pattern().items():
        assert bijective, name
        for s, a, b in steps:
            if s < 16:
                assert a == 1 and b == 1, (name, s, a, b)
            else:
                assert a <= 2 and b <= 2, (name, s, a, b)
