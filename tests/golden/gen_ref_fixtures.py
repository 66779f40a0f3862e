#!/usr/bin/env python3
"""Generate reference-pinned fixtures by RUNNING the reference's own host code under node 12.

What runs (read from /root/reference at generation time, materialised only in a temp dir,
never copied into this repository):
  * src/packing.ts, src/ply.ts, src/mylib.ts  -- TypeScript; type annotations are erased by
    the small eraser below (no tsc exists in this image), then run as ES modules.
  * wgpu-matrix 2.9.1 -- the only copy is sourcesContent[5] of public/main.js.map (SURVEY "WM").

What is written (data only) into tests/golden/:
  * layout.json          -- record sizes for SH degree 0..3 and member byte offsets of the
                            Gaussian record (src/ply.ts:249-257) and the 160-B uniform block
                            (src/renderer.ts:24-33), found by packing sentinel values.
  * <scene>.aos.bin      -- PackedGaussians.gaussiansBuffer for public/{simple,pc_short,m3splat}.ply
  * ply_meta.json        -- numGaussians, nShCoeffs, sha256 of each AoS, min_pos/max_pos.
  * ply_synth/          -- edge-case .ply inputs written here, with PackedGaussians output (or
                          the error it throws) for each: <name>.aos.bin, meta.json.
  * cameras.json         -- wgpu-matrix lookAt/perspective/inverse outputs (Float32 bits) and
                            cam.json-derived view/proj through camera.ts's formulas.

Usage:  python3 tests/golden/gen_ref_fixtures.py   (needs /root/reference and node >= 12)
"""
import hashlib
import json
import os
import re
import shutil
import subprocess
import sys
import tempfile

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))


# ----------------------------------------------------------------------------- TS eraser
def _tokenize(src):
    """Split TS source into tokens; whitespace/comments are kept as 'ws' tokens."""
    toks = []
    i, n = 0, len(src)
    prev_sig = None  # previous significant token text (for regex detection)
    while i < n:
        c = src[i]
        if c in " \t\r\n":
            j = i
            while j < n and src[j] in " \t\r\n":
                j += 1
            toks.append(("ws", src[i:j])); i = j; continue
        if src.startswith("//", i):
            j = src.find("\n", i)
            j = n if j < 0 else j
            toks.append(("ws", src[i:j])); i = j; continue
        if src.startswith("/*", i):
            j = src.find("*/", i + 2) + 2
            toks.append(("ws", src[i:j])); i = j; continue
        if c in "'\"":
            j = i + 1
            while src[j] != c:
                j += 2 if src[j] == "\\" else 1
            toks.append(("str", src[i:j + 1])); i = j + 1; prev_sig = "str"; continue
        if c == "`":
            j, depth = i + 1, 0
            while True:
                if src[j] == "\\":
                    j += 2; continue
                if depth == 0 and src[j] == "`":
                    break
                if src.startswith("${", j):
                    depth += 1; j += 2; continue
                if depth and src[j] == "}":
                    depth -= 1
                j += 1
            toks.append(("str", src[i:j + 1])); i = j + 1; prev_sig = "str"; continue
        if c == "/" and (prev_sig is None or prev_sig in "(,=:[!&|?{};" or prev_sig == "return"):
            j = i + 1
            in_cls = False
            while True:
                if src[j] == "\\":
                    j += 2; continue
                if src[j] == "[":
                    in_cls = True
                elif src[j] == "]":
                    in_cls = False
                elif src[j] == "/" and not in_cls:
                    break
                j += 1
            j += 1
            while j < n and src[j].isalpha():
                j += 1
            toks.append(("re", src[i:j])); i = j; prev_sig = "re"; continue
        if c.isalpha() or c in "_$":
            j = i
            while j < n and (src[j].isalnum() or src[j] in "_$"):
                j += 1
            toks.append(("id", src[i:j])); prev_sig = src[i:j]; i = j; continue
        if c.isdigit() or (c == "." and src[i + 1].isdigit()):
            j = i
            while j < n and (src[j].isalnum() or src[j] in "._"):
                j += 1
            toks.append(("num", src[i:j])); prev_sig = "num"; i = j; continue
        for p in ("||=", "&&=", "===", "!==", "=>", "==", "!=", "<=", ">=", "&&", "||", "++",
                  "--", "+=", "-=", "*=", "/=", "...", "?."):
            if src.startswith(p, i):
                toks.append(("p", p)); prev_sig = p; i += len(p); break
        else:
            toks.append(("p", c)); prev_sig = c; i += 1
    return toks


_OPEN = {"(": ")", "[": "]", "{": "}", "<": ">"}


def _skip_type(toks, k, stops):
    """Return index of the first significant token at depth 0 whose text is in stops."""
    depth = []
    while k < len(toks):
        kind, t = toks[k]
        if kind != "ws":
            if not depth and t in stops:
                return k
            if t in _OPEN:
                depth.append(_OPEN[t])
            elif t == "=>" and depth and depth[-1] == ">":
                pass
            elif depth and t == depth[-1]:
                depth.pop()
        k += 1
    return k


def _next_sig(toks, k):
    while k < len(toks) and toks[k][0] == "ws":
        k += 1
    return k


def _prev_sig(out):
    for kind, t in reversed(out):
        if kind != "ws":
            return t
    return None


def erase_ts(src):
    toks = _tokenize(src)
    out = []
    stack = []  # entries: 'params', 'paren', 'class', 'block', 'bracket'
    pending_class = False
    k = 0
    while k < len(toks):
        kind, t = toks[k]
        top = stack[-1] if stack else None
        if kind == "ws" or kind in ("str", "re", "num"):
            out.append(toks[k]); k += 1; continue
        # statements to drop entirely
        if t == "type" and _prev_sig(out) in (None, ";", "}", "{", "export"):
            j = _skip_type(toks, k + 1, {";"})
            if out and out[-1][1] == "export":
                out.pop()
            elif len(out) >= 2 and out[-2][1] == "export":
                del out[-2:]
            k = j + 1; continue
        if t == "interface":
            j = _next_sig(toks, k + 1)
            j = _skip_type(toks, j + 1, {"{"})
            j = _skip_type(toks, j, {"}"}) if False else j
            depth, m = 0, j
            while True:
                if toks[m][1] == "{": depth += 1
                elif toks[m][1] == "}":
                    depth -= 1
                    if depth == 0: break
                m += 1
            while out and out[-1][1] in ("export",) or (out and out[-1][0] == "ws" and len(out) > 1 and out[-2][1] == "export"):
                out.pop()
            k = m + 1; continue
        if t == "import":
            j = k
            while toks[j][1] != ";":
                j += 1
            stmt = "".join(x[1] for x in toks[k:j + 1])
            m = re.match(r'import\s*\{([^}]*)\}\s*from\s*["\']([^"\']+)["\'];', stmt)
            names = [x.strip() for x in m.group(1).split(",") if x.strip()]
            mod = m.group(2)
            if mod == "wgpu-matrix":
                names = [x for x in names if not x[0].isupper()]
                path = "./wgpu-matrix.mjs"
            else:
                names = [x for x in names if x not in ("NestedData",)]
                path = mod + ".mjs"
            if names:
                out.append(("p", "import { %s } from '%s';" % (", ".join(names), path)))
            k = j + 1; continue
        if t in ("public", "private", "protected", "readonly") and top in ("class", "params"):
            k += 1; continue
        if t == "abstract":
            j = _next_sig(toks, k + 1)
            if toks[j][1] == "class":
                k += 1; continue
            # abstract member: drop through ';'
            while toks[k][1] != ";":
                k += 1
            k += 1; continue
        if t == "as" and _prev_sig(out) not in (None, "{", ",", "import"):
            j = _skip_type(toks, k + 1, {")", "]", ",", ";", "}"})
            k = j; continue
        if t == "class":
            pending_class = True
        if t == "{":
            if pending_class:
                stack.append("class"); pending_class = False
            else:
                stack.append("block")
            out.append(toks[k]); k += 1; continue
        if t == "(":
            # function-like parameter list?
            prev = _prev_sig(out)
            close, depth = k, 0
            while True:
                if toks[close][1] in ("(",): depth += 1
                elif toks[close][1] == ")":
                    depth -= 1
                    if depth == 0: break
                close += 1
            after = _next_sig(toks, close + 1)
            is_params = (top == "class" and prev not in ("=",)) or prev == "function" or \
                (toks[after][1] == "=>") or \
                (prev is not None and len(out) >= 2 and _kw_before(out) == "function")
            if toks[after][1] == ":" and top in ("class", "block", None) and prev not in ("if", "while", "for", "switch"):
                is_params = True
            stack.append("params" if is_params else "paren")
            out.append(toks[k]); k += 1; continue
        if t == "[":
            stack.append("bracket"); out.append(toks[k]); k += 1; continue
        if t in (")", "]", "}"):
            closed = stack.pop() if stack else None
            out.append(toks[k]); k += 1
            if closed == "params":
                j = _next_sig(toks, k)
                if j < len(toks) and toks[j][1] == ":":
                    k = _skip_type(toks, j + 1, {"{", "=>", ";"})
            continue
        if t == ":":
            prev = _prev_sig(out)
            if top == "params" and (prev == "?" or re.match(r"^[\w$]+$", prev or "")):
                if prev == "?":
                    # optional parameter marker
                    for idx in range(len(out) - 1, -1, -1):
                        if out[idx][1] == "?":
                            del out[idx]; break
                k = _skip_type(toks, k + 1, {",", ")", "="}); continue
            if top == "class" and re.match(r"^[\w$]+$", prev or ""):
                j = _skip_type(toks, k + 1, {"=", ";"})
                if toks[j][1] == ";":
                    # declaration without initialiser: drop the member name too
                    while out and out[-1][0] == "ws":
                        out.pop()
                    out.pop()
                    k = j + 1; continue
                k = j; continue
            if _is_decl_colon(out):
                k = _skip_type(toks, k + 1, {"=", ";", ","}); continue
        if t == "||=":
            # a ||= b  ->  a = a || b   (only used on simple lvalues in the reference)
            lhs = []
            for idx in range(len(out) - 1, -1, -1):
                if out[idx][1] in (";", "{", "}") or (out[idx][0] == "ws" and "\n" in out[idx][1]):
                    lhs = out[idx + 1:]; break
            lhs_txt = "".join(x[1] for x in lhs).strip()
            out.append(("p", "= " + lhs_txt + " ||")); k += 1; continue
        out.append(toks[k]); k += 1
    return "".join(x[1] for x in out)


def _kw_before(out):
    sig = [t for kind, t in out if kind != "ws"]
    return sig[-2] if len(sig) >= 2 else None


def _is_decl_colon(out):
    sig = [t for kind, t in out if kind != "ws"]
    return len(sig) >= 2 and sig[-2] in ("let", "const", "var") and re.match(r"^[\w$]+$", sig[-1])


# ----------------------------------------------------------------------------- driver JS
DRIVER = r"""
import fs from 'fs';
import { PackedGaussians } from './ply.mjs';
import { Struct, StaticArray, vec3, vec4, mat4x4, f32 } from './packing.mjs';
import { mat4, mat3, vec3 as wvec3 } from './wgpu-matrix.mjs';

const out = {};
const bits = (arr) => Array.from(new Uint32Array(new Float32Array(arr).buffer));

// Layouts: pack sentinels and locate them.
function offsetsOf(layout, sample) {
  const buf = new ArrayBuffer(layout.size);
  layout.pack(0, sample, new DataView(buf));
  const f = new Float32Array(buf);
  const pos = {};
  for (let i = 0; i < f.length; i++) if (f[i] !== 0) pos[f[i]] = i * 4;
  return [layout.size, pos];
}
const rec = {};
for (const nsh of [1, 4, 9, 16]) {
  const g = new Struct([
    ['position', new vec3(f32)], ['logScale', new vec3(f32)], ['rotQuat', new vec4(f32)],
    ['opacityLogit', f32], ['shCoeffs', new StaticArray(new vec3(f32), nsh)]]);
  const sh = []; for (let k = 0; k < nsh; k++) sh.push([1000 + 3 * k, 1001 + 3 * k, 1002 + 3 * k]);
  const [size, pos] = offsetsOf(g, {position: [1, 2, 3], logScale: [4, 5, 6], rotQuat: [7, 8, 9, 10],
                                    opacityLogit: 11, shCoeffs: sh});
  rec[nsh] = {size, position: pos[1], logScale: pos[4], rotQuat: pos[7], opacityLogit: pos[11],
              sh0: pos[1000], sh1: nsh > 1 ? pos[1003] : null, shLastBlue: pos[1002 + 3 * (nsh - 1)]};
}
const uni = new Struct([
  ['viewMatrix', new mat4x4(f32)], ['projMatrix', new mat4x4(f32)], ['cameraPosition', new vec3(f32)],
  ['tanHalfFovX', f32], ['tanHalfFovY', f32], ['focalX', f32], ['focalY', f32], ['scaleModifier', f32]]);
const m = (b) => [[b, b + 1, b + 2, b + 3], [b + 4, b + 5, b + 6, b + 7], [b + 8, b + 9, b + 10, b + 11], [b + 12, b + 13, b + 14, b + 15]];
const [usize, upos] = offsetsOf(uni, {viewMatrix: m(100), projMatrix: m(200), cameraPosition: [300, 301, 302],
  tanHalfFovX: 400, tanHalfFovY: 401, focalX: 402, focalY: 403, scaleModifier: 404});
out.layout = {record: rec, uniforms: {size: usize, viewMatrix: upos[100], view_m01: upos[101], view_m10: upos[104],
  projMatrix: upos[200], cameraPosition: upos[300], tanHalfFovX: upos[400], tanHalfFovY: upos[401],
  focalX: upos[402], focalY: upos[403], scaleModifier: upos[404]}};

// PLY ingest through PackedGaussians (src/ply.ts).
out.ply = {};
for (const name of ['simple', 'pc_short', 'm3splat']) {
  const b = fs.readFileSync(process.argv[2] + '/public/' + name + '.ply');
  const ab = b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength);
  const g = new PackedGaussians(ab);
  fs.writeFileSync(process.argv[3] + '/' + name + '.aos.bin', Buffer.from(g.gaussiansBuffer));
  out.ply[name] = {numGaussians: g.numGaussians, nShCoeffs: g.nShCoeffs, shDegree: g.sphericalHarmonicsDegree,
                   bytes: g.gaussiansBuffer.byteLength, min_pos: Array.from(g.min_pos), max_pos: Array.from(g.max_pos)};
}

// Synthetic edge-case PLYs (written by gen_ref_fixtures.py) through the same PackedGaussians.
out.ply_synth = {};
for (const f of fs.readdirSync(process.argv[4]).sort()) {
  if (!f.endsWith('.ply')) continue;
  const name = f.slice(0, -4);
  const b = fs.readFileSync(process.argv[4] + '/' + f);
  const ab = b.buffer.slice(b.byteOffset, b.byteOffset + b.byteLength);
  try {
    const g = new PackedGaussians(ab);
    fs.writeFileSync(process.argv[3] + '/synth_' + name + '.aos.bin', Buffer.from(g.gaussiansBuffer));
    out.ply_synth[name] = {numGaussians: g.numGaussians, nShCoeffs: g.nShCoeffs, shDegree: g.sphericalHarmonicsDegree,
                           bytes: g.gaussiansBuffer.byteLength, min_pos: Array.from(g.min_pos), max_pos: Array.from(g.max_pos)};
  } catch (e) {
    out.ply_synth[name] = {error: String(e)};
  }
}

// Cameras through wgpu-matrix (WM) and camera.ts's formulas (src/camera.ts:19-42, :101-138, :467-503).
function getProjectionMatrix(znear, zfar, fovX, fovY) {
  const tanHalfFovY = Math.tan(fovY / 2), tanHalfFovX = Math.tan(fovX / 2);
  const top = tanHalfFovY * znear, bottom = -top, right = tanHalfFovX * znear, left = -right;
  const P = mat4.create();
  P[0] = (2.0 * znear) / (right - left); P[5] = (2.0 * znear) / (top - bottom);
  P[8] = (right + left) / (right - left); P[9] = (top + bottom) / (top - bottom);
  P[10] = zfar / (zfar - znear); P[11] = -(zfar * znear) / (zfar - znear); P[14] = 1.0; P[15] = 0.0;
  return mat4.transpose(P);
}
const focal2fov = (focal, pixels) => 2 * Math.atan(pixels / (2 * focal));
out.cameras = [];
const lookats = [
  {name: 'bench', eye: [0, 0, 0], target: [0, 0, -1]},
  {name: 'app_default', eye: [0, -5, 3], target: [0, 0, 0]},
  {name: 'ref_default_ctor', eye: [0, 0, -5], target: [0, 0, 0]},
];
for (const sc of ['simple', 'pc_short', 'm3splat']) {
  const mn = out.ply[sc].min_pos, mx = out.ply[sc].max_pos;
  const c = wvec3.scale(wvec3.add(mn, mx), 0.5);     // src/index.ts:122-125
  lookats.push({name: sc + '_app', eye: [0, -5, 3], target: Array.from(c)});
  lookats.push({name: sc + '_close', eye: [c[0] + 0.05, c[1] + 0.1, c[2] + 0.6], target: Array.from(c)});
  lookats.push({name: sc + '_behind', eye: [c[0] - 0.1, c[1] - 0.05, c[2] - 0.7], target: Array.from(c)});
}
const sizes = [[256, 256], [1280, 720], [1920, 1080], [3840, 2160], [96, 64]];
for (const L of lookats) for (const [W, H] of sizes) {
  const view = mat4.lookAt(L.eye, L.target, [0, 1, 0]);
  const proj = mat4.perspective(1.04719755, W / H, 0.03, 1000);
  const pos = mat4.getTranslation(mat4.inverse(view));
  out.cameras.push({name: L.name, kind: 'lookat', W, H, eye: L.eye, target: L.target,
                    view: bits(view), proj: bits(proj), campos: bits(pos)});
}
const cams = JSON.parse(fs.readFileSync(process.argv[2] + '/public/cam.json', 'utf8'));
for (const ci of [0, 1, 100, 364]) for (const [W, H] of [[1920, 1080], [256, 256]]) {
  const rc = cams[ci];
  const fovX = focal2fov(rc.fx, W), fovY = focal2fov(rc.fy, H);
  const proj = getProjectionMatrix(0.2, 100, fovX, fovY);
  const R = mat3.create(...rc.rotation.flat());
  const camToWorld = mat4.fromMat3(R);
  mat4.translate(camToWorld, wvec3.mulScalar(rc.position, -1), camToWorld);
  const pos = mat4.getTranslation(mat4.inverse(camToWorld));
  out.cameras.push({name: 'camjson_' + ci, kind: 'json', W, H, json: rc, view: bits(camToWorld), proj: bits(proj),
                    campos: bits(pos)});
}
fs.writeFileSync(process.argv[3] + '/driver_out.json', JSON.stringify(out));
"""


def write_synth_plys(d):
    """Edge-case binary PLY inputs (deterministic); the reference's PackedGaussians parses each."""
    import random
    import struct
    rnd = random.Random(7)
    os.makedirs(d, exist_ok=True)

    def ply(name, props, rows, count=None, extra_header="", eol="\n", trunc=0):
        hdr = ["ply", "format binary_little_endian 1.0", "element vertex %d" % (len(rows) if count is None else count)]
        hdr += ["property %s %s" % (t, n) for t, n in props]
        hdr += [x for x in extra_header.split("|") if x]
        hdr += ["end_header"]
        body = b""
        for row in rows:
            for (t, _), v in zip(props, row):
                if t == "float":
                    body += struct.pack("<f", v)
                elif t == "uchar":
                    body += struct.pack("<B", int(v) & 255)
                elif t == "double":
                    body += struct.pack("<d", v)
        blob = (eol.join(hdr) + eol).encode() + body + b"\0" * 64
        if trunc:
            blob = blob[:len(blob) - 64 - trunc]
        open(os.path.join(d, name + ".ply"), "wb").write(blob)

    def gauss_props(n_rest, extra=()):
        p = [("float", "x"), ("float", "y"), ("float", "z"), ("float", "nx"), ("float", "ny"), ("float", "nz")]
        p += list(extra)
        p += [("float", "f_dc_%d" % c) for c in range(3)]
        p += [("float", "f_rest_%d" % k) for k in range(n_rest)]
        p += [("float", "opacity")] + [("float", "scale_%d" % k) for k in range(3)]
        p += [("float", "rot_%d" % k) for k in range(4)]
        return p

    def row(props):
        out = []
        for t, n in props:
            if t == "uchar":
                out.append(rnd.randrange(256))
            elif n.startswith("scale"):
                out.append(rnd.uniform(-6, -1))
            elif n.startswith("rot"):
                out.append(rnd.gauss(0, 1))
            elif n.startswith("f_rest"):
                out.append(rnd.gauss(0, 0.2))
            else:
                out.append(rnd.uniform(-2, 2))
        return out

    for deg, nr in ((0, 0), (1, 9), (2, 24)):
        pr = gauss_props(nr)
        ply("deg%d" % deg, pr, [row(pr) for _ in range(40)])
    pr = gauss_props(24, extra=(("uchar", "red"), ("uchar", "green"), ("uchar", "blue")))
    ply("deg2_uchar_rgb", pr, [row(pr) for _ in range(33)])
    pr = gauss_props(45)
    pr = [("uchar", n) if n in ("opacity", "rot_0", "f_dc_1") else (t, n) for t, n in pr]
    ply("uchar_mix", pr, [row(pr) for _ in range(25)])
    pr = gauss_props(45)
    rows = [row(pr) for _ in range(12)]
    ri = [i for i, (_, n) in enumerate(pr) if n.startswith("rot")]
    si = [i for i, (_, n) in enumerate(pr) if n.startswith("scale")]
    quats = [(0, 0, 0, 0), (-0.0, 0, 0, 0), (1, 0, 0, 0), (0, 0, 0, -1), (1e-30, 0, 0, 0), (3e38, 3e38, 0, 0),
             (float("nan"), 1, 0, 0), (0, -0.0, -0.0, 1), (2, 0, 0, 0), (float("inf"), 0, 0, 0),
             (-1, -1, -1, -1), (0.5, 0.5, 0.5, 0.5)]
    for r, q in zip(rows, quats):
        for i, v in zip(ri, q):
            r[i] = v
    rows[3][si[0]] = 100.0
    rows[4][si[1]] = float("nan")
    rows[5][0] = float("nan")
    ply("quat_scale_edge", pr, rows)
    pr = gauss_props(45)
    pr = pr[-4:] + pr[-8:-4] + pr[6:-8] + pr[:6]
    ply("reordered", pr, [row(pr) for _ in range(20)])
    pr = gauss_props(45)
    pr2 = pr[:3] + [("double", "weight")] + pr[3:]
    ply("double_prop", pr2, [row(pr2) for _ in range(10)])
    pr = gauss_props(45)
    ply("face_element", pr, [row(pr) for _ in range(10)],
        extra_header="element face 0|property list uchar int vertex_indices")
    pr = gauss_props(45)
    pr2 = pr[:3] + [("float", "7")] + pr[3:]
    ply("integer_name", pr2, [row(pr2) for _ in range(10)])
    pr = gauss_props(5)
    ply("bad_degree", pr, [row(pr) for _ in range(4)])
    pr = gauss_props(45)
    ply("crlf", pr, [row(pr) for _ in range(8)], eol="\r\n")
    pr = gauss_props(45)
    ply("truncated", pr, [row(pr) for _ in range(8)], trunc=100)
    pr = gauss_props(45)
    ply("zero_vertices", pr, [])


def main():
    if not os.path.isdir(REF):
        sys.exit("reference not present; fixtures are committed, nothing to do")
    tmp = tempfile.mkdtemp(prefix="gsref_")
    try:
        smap = json.load(open(os.path.join(REF, "public/main.js.map")))
        wm = smap["sourcesContent"][5]
        assert wm.startswith("/* wgpu-matrix@2.9.1"), wm[:40]
        open(os.path.join(tmp, "wgpu-matrix.mjs"), "w").write(wm)
        for name in ("packing", "ply", "mylib"):
            js = erase_ts(open(os.path.join(REF, "src", name + ".ts")).read())
            open(os.path.join(tmp, name + ".mjs"), "w").write(js)
        open(os.path.join(tmp, "driver.mjs"), "w").write(DRIVER)
        outdir = os.path.join(tmp, "out")
        os.makedirs(outdir)
        synth = os.path.join(HERE, "ply_synth")
        write_synth_plys(synth)
        r = subprocess.run(["node", "--experimental-modules", "--no-warnings", "driver.mjs", REF, outdir, synth],
                           cwd=tmp, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            sys.exit("node driver failed (temp dir kept: %s)" % tmp)
        res = json.load(open(os.path.join(outdir, "driver_out.json")))
        for name in res["ply"]:
            blob = open(os.path.join(outdir, name + ".aos.bin"), "rb").read()
            res["ply"][name]["sha256"] = hashlib.sha256(blob).hexdigest()
            shutil.copy(os.path.join(outdir, name + ".aos.bin"), os.path.join(HERE, name + ".aos.bin"))
        json.dump(res["layout"], open(os.path.join(HERE, "layout.json"), "w"), indent=1, sort_keys=True)
        json.dump(res["ply"], open(os.path.join(HERE, "ply_meta.json"), "w"), indent=1, sort_keys=True)
        for name, m in res["ply_synth"].items():
            if "error" not in m:
                blob = open(os.path.join(outdir, "synth_" + name + ".aos.bin"), "rb").read()
                m["sha256"] = hashlib.sha256(blob).hexdigest()
                shutil.copy(os.path.join(outdir, "synth_" + name + ".aos.bin"), os.path.join(synth, name + ".aos.bin"))
        json.dump(res["ply_synth"], open(os.path.join(synth, "meta.json"), "w"), indent=1, sort_keys=True)
        json.dump(res["cameras"], open(os.path.join(HERE, "cameras.json"), "w"))
        print("fixtures written to", HERE)
    finally:
        if os.environ.get("KEEP_TMP") is None:
            shutil.rmtree(tmp, ignore_errors=True)
        else:
            print("temp dir:", tmp)


if __name__ == "__main__":
    main()
