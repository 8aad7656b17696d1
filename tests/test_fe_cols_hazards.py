"""Static check of the generated field-product columns (ouroboros-consensus_amd/csrc/fe_cols.hpp):
every carry a `v_mad_u64_u32` writes (VCC or an SGPR pair) is read by a `v_addc_co_u32` /
`v_cndmask_b32_e64` of the same asm block only after at least two wait states -- the gfx950
rule the generator (tools/gen_fe_cols.py) schedules for instead of `s_nop` padding -- and no
block reads a carry it did not write itself (nothing is carried across blocks)."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "ouroboros-consensus_amd", "csrc", "fe_cols.hpp")


def _blocks():
    text = open(HDR).read()
    for m in re.finditer(r'asm\("((?:[^"\\]|\\.)*)"', text):
        yield [ins.strip() for ins in m.group(1).split("\\n\\t")]


def _wait_states(ins):
    m = re.match(r"s_nop (\d+)$", ins)
    return int(m.group(1)) + 1 if m else 1


def test_carry_reads_are_two_wait_states_after_their_writes():
    nblocks = nreads = 0
    for block in _blocks():
        nblocks += 1
        written = {}                      # carry register -> issue clock of its last write
        # (each instruction advances the clock by 1, s_nop N by N + 1: the wait states between a
        # write at w and a read at r are r - w - 1)
        clock = 0
        for ins in block:
            op, _, args = ins.partition(" ")
            a = [x.strip() for x in args.split(",")] if args else []
            if op == "v_mad_u64_u32":
                written[a[1]] = clock
            elif op == "v_addc_co_u32":
                cin = a[4]
                assert cin in written, (ins, block)
                assert clock - written[cin] >= 3, (ins, block)   # >= 2 wait states in between
                nreads += 1
                written[a[1]] = clock     # the carry-out rewrites the register
            elif op == "v_cndmask_b32_e64":
                sel = a[3]
                assert sel in written, (ins, block)
                assert clock - written[sel] >= 3, (ins, block)
                nreads += 1
            else:
                assert op == "s_nop", ins
            clock += _wait_states(ins)
    assert nblocks > 40 and nreads > 250


def test_only_small_columns_keep_padding():
    # one-product columns of one or two MACs and two-product columns of one MAC per product
    for block in _blocks():
        nmad = sum(ins.startswith("v_mad_u64_u32") for ins in block)
        nops = [ins for ins in block if ins.startswith("s_nop")]
        pair = any("%1, " in ins and ins.startswith("v_mad_u64_u32 %1") for ins in block)
        if nops:
            assert (pair and nmad == 2) or (not pair and nmad <= 2), block
