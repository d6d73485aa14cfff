"""ISA of the level-0 packet traversal's dependent step (k_trace_pkt<COUNT=0, GEN=1, MINW=8>, the
kernel that traces every primary ray of a frame): one internal-node step of the sign-specialised
node loop (SGN 0) and one triangle of the leaf loop, per basic block, with the instruction-class
counts of the step's paths.  Compiles trace.hip for gfx950 to assembly (device only, the
Makefile's flags) -- no GPU needed.

usage: python tools/isa_steps.py [out.txt]"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNEL = "_ZN4pgrt11k_trace_pktILb0ELb1ELi8ELb0EE"


def classify(ins):
    op = ins.split()[0]
    if op.startswith("s_load") or op.startswith("s_buffer_load"):
        return "SMEM"
    if op.startswith("ds_"):
        return "LDS"
    if op.startswith(("global_", "buffer_", "flat_")):
        return "VMEM"
    if op.startswith("s_waitcnt"):
        return "WAIT"
    if op.startswith(("s_cbranch", "s_branch")):
        return "BRANCH"
    if op.startswith("s_nop"):
        return "NOP"
    if op.startswith("s_"):
        return "SALU"
    if op.startswith("v_"):
        return "VALU"
    return "OTHER"


def blocks(lines):
    """[(label, [instructions])] of a function body, in layout order."""
    out, cur, name = [], [], "entry"
    for ln in lines:
        s = ln.split(";")[0].strip()
        m = re.match(r"^(\.LBB\d+_\d+|%bb\.\d+):?", ln.strip())
        if m or ln.strip().startswith("; %bb."):
            out.append((name, cur))
            name = m.group(1) if m else ln.strip()[2:].split(":")[0]
            cur = []
            continue
        if not s or s.startswith(".") or s.endswith(":"):
            continue
        cur.append(s)
    out.append((name, cur))
    return out


def counts(ins):
    c = {}
    for i in ins:
        k = classify(i)
        c[k] = c.get(k, 0) + 1
    return c


def main():
    out_path = sys.argv[1] if len(sys.argv) > 1 else None
    src = os.path.join(ROOT, "pgi_raytracing_amd", "csrc", "trace.hip")
    with tempfile.TemporaryDirectory() as td:
        asm = os.path.join(td, "trace.s")
        subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off",
                        "-fhip-fp32-correctly-rounded-divide-sqrt", "-I" + os.path.join(ROOT, "include"),
                        "-I" + os.path.join(ROOT, "pgi_raytracing_amd", "csrc"), "-mllvm", "-disable-machine-licm",
                        "--offload-device-only", "-S", "-o", asm, src], check=True, capture_output=True)
        text = open(asm).read().splitlines()
    start = next(i for i, l in enumerate(text) if l.startswith(KERNEL) and l.split(";")[0].rstrip().endswith(":"))
    end = next(i for i in range(start + 1, len(text)) if text[i].startswith(".Lfunc_end"))
    bl = blocks(text[start + 1:end])
    names = [b[0] for b in bl]
    rep = []
    # the first sign-specialised node loop: the loop header whose block reads the stack top (LDS)
    # and issues the node's scalar loads at offsets 0x0 / 0x20 / 0x30
    hdr = next(k for k, (n, ins) in enumerate(bl) if any(i.startswith("ds_read_b32") for i in ins)
               and any(re.match(r"s_load_dwordx8 .*offset:0x0$", i) for i in ins)
               and any(re.match(r"s_load_dword\w* .*offset:0x30$", i) for i in ins))
    # the loop's blocks: from the header to the block that branches back to it
    back = next(k for k in range(hdr, len(bl)) if any(i.split()[0] == "s_branch" and i.split()[1] == bl[hdr][0]
                                                       for i in bl[k][1]))
    node_blocks = bl[hdr:back + 1]
    rep.append(f"k_trace_pkt<COUNT=0, GEN=1, MINW=8> ({KERNEL}...): internal-node step, SGN 0 loop "
               f"(blocks {node_blocks[0][0]} .. {node_blocks[-1][0]})")
    tot = {}
    for n, ins in node_blocks:
        c = counts(ins)
        for k, v in c.items():
            tot[k] = tot.get(k, 0) + v
        rep.append(f"  -- {n}: {len(ins)} instructions {dict(sorted(c.items()))}")
        rep += ["       " + i for i in ins]
    head = counts(node_blocks[0][1])
    rep.append(f"  header block (every step: stack-top read, node loads, wait, both box tests, ballots): "
               f"{dict(sorted(head.items()))}")
    rep.append(f"  all blocks of the loop (the three child cases are alternatives): {dict(sorted(tot.items()))}")
    # the leaf loop: the loop header with the triangle's scalar loads (offset 0x0 / 0x20 from one
    # base, Ng from another) -- the first such header after the node loops
    leaf = next(k for k, (n, ins) in enumerate(bl) if k > back and
                sum(1 for i in ins if i.startswith("s_load_dword")) == 3 and
                not any(i.startswith("ds_") or "offset:0x30" in i for i in ins) and
                any(re.match(r"s_load_dwordx8 .*offset:0x0$", i) for i in ins) and
                any(re.match(r"s_load_dwordx4 .*offset:0x20$", i) for i in ins))
    rep.append("")
    rep.append(f"leaf loop, one triangle (tri_test_ng against every lane's ray): from {bl[leaf][0]}")
    k = leaf
    seen = 0
    while k < len(bl) and seen < 4:  # the header and the edge / depth tests up to the division
        n, ins = bl[k]
        c = counts(ins)
        rep.append(f"  -- {n}: {len(ins)} instructions {dict(sorted(c.items()))}")
        rep += ["       " + i for i in ins]
        if any("v_div_scale" in i for i in ins):
            break
        k += 1
        seen += 1
    txt = "\n".join(rep)
    print(txt)
    if out_path:
        with open(out_path, "w") as f:
            f.write(txt + "\n")


if __name__ == "__main__":
    main()
