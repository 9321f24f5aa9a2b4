"""Inline-asm clobber audit of the engine's device code (one pass over every
translation unit).

Round 2 found a hang whose cause was an inline-asm string that wrote SCC
(`s_or_b64`) without declaring it: the compiler kept a loop's exit condition
in SCC across the statement ("k_verify_main never left its loop").
This tool preprocesses every source with hipcc -E (so the macro-built
templates -- COA_CHAIN8, COA_RARE_BEGIN, ... -- are expanded exactly as
compiled), finds every asm statement and checks that each implicit register
its template writes is in its clobber list (or bound as an output operand):

  vcc   carry-out VOP2/VOPC forms (v_add_co/v_addc/v_sub_co/v_subb *_e32,
        v_cmp*_e32), or vcc named as a destination
  scc   SALU arithmetic, logic, shifts and compares (s_add, s_or, s_cmp, ...)
  exec  *saveexec*, v_cmpx*, or exec named as a destination

usage: python tools/asm_audit.py [files...]   (default: every csrc file with asm)
Exit 1 and one line per finding when a clobber is missing.
"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "xrpl-coa-prototype_amd", "csrc")

# SALU instructions that do NOT write SCC
SCC_SAFE = re.compile(r"^s_(nop|waitcnt|branch|cbranch_\w+|setprio|sleep|mov_b32|mov_b64|getpc_b64|barrier|"
                      r"endpgm|sendmsg|dcache_\w+|icache_\w+|ttracedata|trap|setreg\w*|getreg\w*|memtime|memrealtime|"
                      r"load_\w+|buffer_load_\w+|store_\w+)$")


def _strings(expr):
    """Concatenated contents of the C string literals in an expression."""
    out = []
    for m in re.finditer(r'"((?:[^"\\]|\\.)*)"', expr):
        out.append(bytes(m.group(1), "utf-8").decode("unicode_escape"))
    return "".join(out)


def _split_top(s, sep):
    """Split s at top-level occurrences of sep (outside parentheses/strings)."""
    parts, depth, cur, i, instr = [], 0, [], 0, False
    while i < len(s):
        c = s[i]
        if c == '"':
            j = i + 1
            while j < len(s) and s[j] != '"':
                j += 2 if s[j] == "\\" else 1
            cur.append(s[i:j + 1])
            i = j + 1
            continue
        if c in "([{":
            depth += 1
        elif c in ")]}":
            depth -= 1
        if c == sep and depth == 0:
            parts.append("".join(cur))
            cur = []
        else:
            cur.append(c)
        i += 1
    parts.append("".join(cur))
    return parts


def asm_statements(text):
    """(template, outputs, clobbers) of every asm statement in preprocessed C++."""
    for m in re.finditer(r"\basm\b\s*(?:volatile\s*|__volatile__\s*)?\(", text):
        i, depth = m.end(), 1
        j = i
        while depth and j < len(text):
            if text[j] == '"':
                k = j + 1
                while text[k] != '"':
                    k += 2 if text[k] == "\\" else 1
                j = k + 1
                continue
            depth += {"(": 1, ")": -1}.get(text[j], 0)
            j += 1
        body = text[i:j - 1]
        parts = _split_top(body, ":")
        tmpl = _strings(parts[0])
        outputs = parts[1] if len(parts) > 1 else ""
        clobbers = set(_strings(x) for x in re.findall(r'"[^"]*"', parts[3])) if len(parts) > 3 else set()
        yield tmpl, outputs, clobbers, text[:m.start()].count("\n") + 1


def writes(tmpl):
    """Implicit registers an asm template writes."""
    found = set()
    for line in re.split(r"[\n;]", tmpl):
        line = line.strip()
        if not line or line.endswith(":") or line.startswith("."):
            continue
        op = line.split()[0]
        args = line[len(op):]
        dst = args.split(",")[0].strip() if args.strip() else ""
        if re.match(r"v_(add|sub|subrev)_co_u32_e32|v_(addc|subb|subbrev)_co_u32_e32|v_cmp\w*_e32", op):
            found.add("vcc")
        if re.match(r"v_(add|sub|subrev|addc|subb)_co\w*_e64|v_mad_u64_u32|v_mad_i64_i32|v_div_scale", op):
            # e64 forms write an explicit SGPR pair: vcc only if named
            if re.search(r",\s*vcc\b", args.split(",", 2)[1] if args.count(",") >= 1 else ""):
                found.add("vcc")
        if dst in ("vcc", "vcc_lo", "vcc_hi"):
            found.add("vcc")
        if op.startswith("s_") and not SCC_SAFE.match(op):
            found.add("scc")
        if "saveexec" in op or op.startswith("v_cmpx") or dst in ("exec", "exec_lo", "exec_hi"):
            found.add("exec")
    return found


def audit(path):
    cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-std=c++17", "-E", "-I" + os.path.join(ROOT, "include"),
           "--cuda-device-only", "-x", "hip", path]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError(f"hipcc -E failed for {path}: {r.stderr[-2000:]}")
    issues, n = [], 0
    seen = set()
    for tmpl, outputs, clobbers, line in asm_statements(r.stdout):
        key = (tmpl, tuple(sorted(clobbers)), outputs)
        if key in seen:  # the same inlined statement from one header
            continue
        seen.add(key)
        n += 1
        for reg in sorted(writes(tmpl)):
            if reg in clobbers or re.search(r'"=[^"]*\{?' + reg, outputs):
                continue
            first = next((l.strip() for l in tmpl.splitlines() if l.strip()), "")
            issues.append(f"{os.path.basename(path)}: asm writes {reg} without a clobber: {first[:70]}")
    return n, issues


def sources():
    out = []
    for f in sorted(os.listdir(CSRC)):
        if f.endswith(".hip"):
            out.append(os.path.join(CSRC, f))
    return out


def main(argv):
    files = argv or sources()
    total, bad = 0, []
    for f in files:
        n, issues = audit(f)
        total += n
        bad += issues
    for b in sorted(set(bad)):
        print(b)
    print(f"asm audit: {total} distinct asm statements in {len(files)} files, {len(set(bad))} missing clobbers")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
