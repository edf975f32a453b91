#!/usr/bin/env python3
"""The Rust `extern "C"` binding of include/pktgpu.h that INTEGRATION.md carries, and the C/Rust
declaration parsers tests/test_rust_binding.py uses to check it field by field and argument by
argument.  (No cargo in this image: the binding cannot be compiled here, so it is checked
mechanically against the header instead.)

  python scripts/rust_binding.py           # print the binding generated from the header
  python scripts/rust_binding.py --update  # rewrite INTEGRATION.md's block from the header
"""
import os
import re

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(REPO, "include", "pktgpu.h")

C_SCALARS = {"uint8_t": "u8", "uint16_t": "u16", "uint32_t": "u32", "uint64_t": "u64", "int32_t": "i32",
             "int": "c_int", "float": "f32", "size_t": "usize", "char": "c_char", "void": "c_void",
             "pkt_ctx_t": "PktCtx", "pkt_batch_t": "PktBatch", "pkt_out_t": "PktOut", "pkt_chain_t": "PktChain",
             "pkt_field_spec_t": "PktFieldSpec", "pkt_gen_field_t": "PktGenField", "pkt_gen_t": "PktGen",
             "pkt_mgpu_t": "PktMgpu", "pkt_gather_piece_t": "PktGatherPiece", "pkt_pcap_stream_t": "PktPcapStream"}
STRUCTS = {"pkt_batch": "PktBatch", "pkt_out": "PktOut", "pkt_field_spec": "PktFieldSpec", "pkt_chain": "PktChain",
           "pkt_gen_field": "PktGenField", "pkt_gather_piece": "PktGatherPiece"}


def _strip(src):
    return re.sub(r"/\*.*?\*/", "", src, flags=re.S)


def c_type(decl):
    """'const uint64_t *const *values' -> ('u64', ['const', 'const']): the Rust base type and the
    mutability of what each pointer level points to, innermost first.  An array parameter
    (`uint64_t off[2]`) is a pointer."""
    decl = decl.strip()
    is_arr = bool(re.search(r"\[[^\]]*\]\s*$", decl))
    decl = re.sub(r"\[[^\]]*\]\s*$", "", decl).strip()
    toks = re.findall(r"\*|const|[A-Za-z_][A-Za-z0-9_]*", decl)
    idents = [i for i, t in enumerate(toks) if t not in ("*", "const")]
    if len(idents) >= 2:  # the declarator's name
        del toks[idents[-1]]
    if is_arr:
        toks.append("*")
    base, levels, c = None, [], False
    for t in toks:
        if t == "const":
            c = True
        elif t == "*":
            levels.append("const" if c else "mut")
            c = False
        else:
            base = t
    return C_SCALARS[base], levels


def rust_of(base, levels):
    s = base
    for q in levels:  # innermost pointer first
        s = f"*{q} {s}"
    return s


def header_structs():
    src = _strip(open(HEADER).read())
    out = {}
    for m in re.finditer(r"typedef struct (\w+) \{(.*?)\}\s*\w+;", src, flags=re.S):
        name = m.group(1)
        if name not in STRUCTS:
            continue
        fields = []
        for line in m.group(2).split(";"):
            line = line.strip()
            if not line:
                continue
            fname = re.findall(r"[A-Za-z_][A-Za-z0-9_]*", line)[-1]
            fields.append((fname, rust_of(*c_type(line))))
        out[STRUCTS[name]] = fields
    return out


def header_functions():
    src = _strip(open(HEADER).read())
    src = re.sub(r"#.*", "", src)
    out = {}
    for m in re.finditer(r"([A-Za-z_][A-Za-z0-9_ \*]*?)\b(pkt_[a-z0-9_]+)\s*\(([^)]*)\)\s*;", src):
        ret, name, params = m.group(1), m.group(2), m.group(3).strip()
        ret = ret.replace("typedef", "").strip()
        args = []
        if params and params != "void":
            for p in params.split(","):
                pname = re.findall(r"[A-Za-z_][A-Za-z0-9_]*", re.sub(r"\[.*\]", "", p))[-1]
                args.append((pname, rust_of(*c_type(p))))
        r = rust_of(*c_type(ret + " x")) if ret != "void" else None
        out[name] = (args, r)
    return out


def generate():
    st, fn = header_structs(), header_functions()
    lines = ["// src/gpu.rs — packet_rs's batched GPU decode through libpktgpu (include/pktgpu.h, ABI v5).",
             "// Every struct and function of the header, field for field (tests/test_rust_binding.py).",
             "#![allow(non_camel_case_types, dead_code)]",
             "use std::os::raw::{c_char, c_int, c_void};", ""]
    for name, fields in st.items():
        lines.append("#[repr(C)]")
        lines.append(f"#[derive(Clone, Copy)] pub struct {name} {{")
        for f, t in fields:
            lines.append(f"    pub {f}: {t},")
        lines.append("}")
    for opaque in ("PktCtx", "PktGen", "PktMgpu"):
        lines.append(f"#[repr(C)] pub struct {opaque} {{ _p: [u8; 0] }}")
    lines += ["", '#[link(name = "pktgpu")]', 'extern "C" {']
    for name, (args, ret) in fn.items():
        a = ", ".join(f"{n}: {t}" for n, t in args)
        r = f" -> {ret}" if ret else ""
        lines.append(f"    pub fn {name}({a}){r};")
    lines.append("}")
    return "\n".join(lines)


RUST_BLOCK = re.compile(r"```rust\n(.*?)```", re.S)


def rust_structs(code):
    out = {}
    for m in re.finditer(r"pub struct (\w+) \{(.*?)\}", code, flags=re.S):
        body = m.group(2)
        if "_p:" in body:
            continue
        out[m.group(1)] = [(f, " ".join(t.split())) for f, t in re.findall(r"pub (\w+):\s*([^,]+),", body)]
    return out


def rust_functions(code):
    out = {}
    for m in re.finditer(r"pub fn (pkt_\w+)\(([^)]*)\)\s*(?:->\s*([^;]+))?;", code):
        args = [(n, " ".join(t.split())) for n, t in re.findall(r"(\w+):\s*([^,]+)", m.group(2))]
        out[m.group(1)] = (args, " ".join(m.group(3).split()) if m.group(3) else None)
    return out




def update_integration():
    """Rewrite the generated part of INTEGRATION.md's ```rust block (up to the helpers)."""
    p = os.path.join(REPO, "INTEGRATION.md")
    md = open(p).read()
    a = md.index("```rust\n") + len("```rust\n")
    b = md.index("\n// ---- safe-ish helpers", a)
    open(p, "w").write(md[:a] + generate() + "\n" + md[b:])


if __name__ == "__main__":
    import sys
    if "--update" in sys.argv:
        update_integration()
    else:
        print(generate())
