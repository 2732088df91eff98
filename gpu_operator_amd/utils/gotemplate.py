"""A small Go ``text/template`` engine with the Sprig/Helm functions our chart uses.

Lets the tests and ``gpuop-cfg validate clusterpolicy`` render the Helm chart
(deployments/amd-gpu-operator) the way ``helm template`` would, without a helm binary — the
reference's config validation renders its chart the same way.

Supported: text/actions with ``{{-``/``-}}`` trimming, comments, pipelines (``|`` passes the
value as the last argument), parenthesised sub-pipelines, ``$``/``.``/``$var`` field chains,
variable declaration/assignment, ``if/else if/else``, ``range`` (lists and maps, with
``$i, $v :=``), ``with/else``, ``define``/``template``/``include``, and the functions in
:data:`FUNCS` (include, toYaml, nindent, indent, quote, squote, printf, default, empty,
trunc, trimSuffix, trimPrefix, replace, lower, upper, list, dict, index, omit, hasKey, and,
or, not, eq, ne, lt, gt, len, required, fail, toString, b64enc, contains).
"""

from __future__ import annotations

import base64
import glob
import re
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------------------------------
# lexing of the template into text / action pieces
# ------------------------------------------------------------------------------------------
_ACTION = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)


def _pieces(src: str) -> List[Tuple[str, str]]:
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip()
        if out and out[-1][0] == "trim_next":
            out.pop()
            text = text.lstrip()
        out.append(("text", text))
        body = m.group(2).strip()
        if body.startswith("/*"):
            out.append(("comment", ""))
        else:
            out.append(("action", body))
        if m.group(3):
            out.append(("trim_next", ""))
        pos = m.end()
    text = src[pos:]
    if out and out[-1][0] == "trim_next":
        out.pop()
        text = text.lstrip()
    out.append(("text", text))
    return [p for p in out if not (p[0] == "text" and p[1] == "") and p[0] != "comment"]


# ------------------------------------------------------------------------------------------
# expression tokens
# ------------------------------------------------------------------------------------------
_TOK = re.compile(r'''\s*(?:
    (?P<str>"(?:\\.|[^"\\])*") |
    (?P<raw>`[^`]*`) |
    (?P<num>-?\d+(?:\.\d+)?) |
    (?P<decl>:=) |
    (?P<assign>=) |
    (?P<pipe>\|) |
    (?P<lp>\() |
    (?P<rp>\)(?:\.[A-Za-z_][\w]*)*) |
    (?P<comma>,) |
    (?P<var>\$[\w]*(?:\.[A-Za-z_][\w]*)*) |
    (?P<field>(?:\.[A-Za-z_][\w]*)+|\.) |
    (?P<ident>[A-Za-z_][\w]*)
)''', re.X)


def _tokens(s: str) -> List[Tuple[str, str]]:
    out = []
    pos = 0
    s = s.strip()
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m or m.end() == pos:
            raise TemplateError(f"cannot tokenize {s[pos:]!r}")
        kind = m.lastgroup
        out.append((kind, m.group(kind)))
        pos = m.end()
    return out


# ------------------------------------------------------------------------------------------
# AST
# ------------------------------------------------------------------------------------------
class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Action(Node):
    def __init__(self, expr):
        self.expr = expr


class If(Node):
    def __init__(self):
        self.branches: List[Tuple[Optional[str], List[Node]]] = []   # (cond expr | None=else, body)


class Range(Node):
    def __init__(self, expr):
        self.expr = expr
        self.body: List[Node] = []
        self.else_: List[Node] = []


class With(Node):
    def __init__(self, expr):
        self.expr = expr
        self.body: List[Node] = []
        self.else_: List[Node] = []


class TemplateCall(Node):
    def __init__(self, expr):
        self.expr = expr


def _parse(pieces: List[Tuple[str, str]], defines: Dict[str, List[Node]]) -> List[Node]:
    root: List[Node] = []
    stack: List[Tuple[Node, List[Node]]] = []   # (control node, current body list)
    cur = root
    for kind, s in pieces:
        if kind == "text":
            cur.append(Text(s))
            continue
        word = s.split(None, 1)[0] if s else ""
        rest = s[len(word):].strip()
        if word == "if":
            n = If()
            n.branches.append((rest, []))
            cur.append(n)
            stack.append((n, cur))
            cur = n.branches[-1][1]
        elif word == "else":
            node, parent = stack[-1]
            if isinstance(node, If):
                cond = rest[3:].strip() if rest.startswith("if ") or rest == "if" else None
                node.branches.append((cond, []))
                cur = node.branches[-1][1]
            else:
                cur = node.else_
        elif word == "range":
            n = Range(rest)
            cur.append(n)
            stack.append((n, cur))
            cur = n.body
        elif word == "with":
            n = With(rest)
            cur.append(n)
            stack.append((n, cur))
            cur = n.body
        elif word == "define":
            name = _unquote(rest)
            body: List[Node] = []
            defines[name] = body
            stack.append((Text(name), cur))   # marker
            cur = body
        elif word == "end":
            if not stack:
                raise TemplateError("unexpected {{end}}")
            _, cur = stack.pop()
        elif word == "template":
            cur.append(TemplateCall(rest))
        else:
            cur.append(Action(s))
    if stack:
        raise TemplateError("unterminated block")
    return root


def _unquote(s: str) -> str:
    s = s.strip()
    if s.startswith('"'):
        return bytes(s[1:-1], "utf-8").decode("unicode_escape")
    if s.startswith("`"):
        return s[1:-1]
    raise TemplateError(f"expected string, got {s!r}")


# ------------------------------------------------------------------------------------------
# evaluation
# ------------------------------------------------------------------------------------------
def truthy(v: Any) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def _field(v: Any, name: str) -> Any:
    if isinstance(v, dict):
        return v.get(name)
    return getattr(v, name, None)


def _to_yaml(v: Any) -> str:
    if v is None:
        return "null"
    s = yaml.safe_dump(v, default_flow_style=False, sort_keys=True, width=10 ** 6)
    if s.endswith("\n...\n"):
        s = s[:-5]
    return s.rstrip("\n")


def _printf(fmt: str, *args) -> str:
    py = re.sub(r"%v", "%s", fmt)
    conv = re.findall(r"%[-+ #0]*\d*(?:\.\d+)?([sdfxXoeEgGq%])", py)
    vals, i = [], 0
    for c in conv:
        if c == "%":
            continue
        a = args[i] if i < len(args) else None
        i += 1
        if c == "q":
            vals.append('"' + _str(a) + '"')
        elif c in "dxXo":
            vals.append(int(a))
        elif c in "feEgG":
            vals.append(float(a))
        else:
            vals.append(_str(a))
    return py.replace("%q", "%s") % tuple(vals) if conv else py


def _str(v: Any) -> str:
    if v is None:
        return ""
    if v is True:
        return "true"
    if v is False:
        return "false"
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    if isinstance(v, (dict, list)):
        return _go_repr(v)
    return str(v)


def _go_repr(v: Any) -> str:
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_repr(x)}" for k, x in sorted(v.items())) + "]"
    if isinstance(v, list):
        return "[" + " ".join(_go_repr(x) for x in v) + "]"
    return _str(v)


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + line for line in _str(s).split("\n"))


def _default(d, v=None):
    return v if truthy(v) else d


def _required(msg, v=None):
    if v is None or v == "":
        raise TemplateError(msg)
    return v


def _fail(msg):
    raise TemplateError(msg)


def _omit(d, *keys):
    return {k: v for k, v in (d or {}).items() if k not in keys}


def _index(v, *keys):
    for k in keys:
        if v is None:
            return None
        v = v[k] if isinstance(v, list) else (v or {}).get(k)
    return v


FUNCS: Dict[str, Callable] = {
    "toYaml": _to_yaml,
    "nindent": lambda n, s: "\n" + _indent(n, s),
    "indent": _indent,
    "quote": lambda *a: " ".join('"' + _str(x).replace("\\", "\\\\").replace('"', '\\"') + '"' for x in a),
    "squote": lambda *a: " ".join("'" + _str(x) + "'" for x in a),
    "printf": _printf,
    "print": lambda *a: "".join(_str(x) for x in a),
    "default": _default,
    "empty": lambda v: not truthy(v),
    "trunc": lambda n, s: _str(s)[: int(n)] if int(n) >= 0 else _str(s)[int(n):],
    "trimSuffix": lambda suf, s: _str(s)[: -len(suf)] if suf and _str(s).endswith(suf) else _str(s),
    "trimPrefix": lambda pre, s: _str(s)[len(pre):] if pre and _str(s).startswith(pre) else _str(s),
    "trim": lambda s: _str(s).strip(),
    "replace": lambda old, new, s: _str(s).replace(old, new),
    "lower": lambda s: _str(s).lower(),
    "upper": lambda s: _str(s).upper(),
    "contains": lambda sub, s: sub in _str(s),
    "hasPrefix": lambda pre, s: _str(s).startswith(pre),
    "list": lambda *a: list(a),
    "dict": lambda *a: {a[i]: a[i + 1] for i in range(0, len(a), 2)},
    "index": _index,
    "omit": _omit,
    "hasKey": lambda d, k: k in (d or {}),
    "keys": lambda d: sorted((d or {}).keys()),
    "and": lambda *a: next((x for x in a if not truthy(x)), a[-1] if a else True),
    "or": lambda *a: next((x for x in a if truthy(x)), a[-1] if a else False),
    "not": lambda v: not truthy(v),
    "eq": lambda a, *b: any(a == x for x in b),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: a < b,
    "gt": lambda a, b: a > b,
    "le": lambda a, b: a <= b,
    "ge": lambda a, b: a >= b,
    "len": lambda v: len(v or []),
    "required": _required,
    "fail": _fail,
    "toString": _str,
    "b64enc": lambda s: base64.b64encode(_str(s).encode()).decode(),
    "int": lambda v: int(v or 0),
}


class Template:
    def __init__(self):
        self.defines: Dict[str, List[Node]] = {}
        self.files: Dict[str, List[Node]] = {}

    def add(self, name: str, src: str) -> None:
        self.files[name] = _parse(_pieces(src), self.defines)

    def render(self, name: str, dot: Any) -> str:
        out: List[str] = []
        self._exec(self.files[name], dot, {"$": dot}, out)
        return "".join(out)

    # -- execution ---------------------------------------------------------------------------
    def _exec(self, nodes: List[Node], dot: Any, vars_: Dict[str, Any], out: List[str]) -> None:
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Action):
                v = self._action(n.expr, dot, vars_)
                if v is not _NOOUT:
                    out.append(_str(v))
            elif isinstance(n, If):
                for cond, body in n.branches:
                    if cond is None or truthy(self._pipeline(cond, dot, vars_)):
                        self._exec(body, dot, dict(vars_), out)
                        break
            elif isinstance(n, With):
                v = self._pipeline(n.expr, dot, vars_)
                if truthy(v):
                    self._exec(n.body, v, dict(vars_), out)
                else:
                    self._exec(n.else_, dot, dict(vars_), out)
            elif isinstance(n, Range):
                self._range(n, dot, vars_, out)
            elif isinstance(n, TemplateCall):
                toks = _tokens(n.expr)
                name = _unquote(toks[0][1])
                arg = self._eval_tokens(toks[1:], dot, vars_) if len(toks) > 1 else None
                out.append(self._include(name, arg))

    def _range(self, n: Range, dot, vars_, out):
        expr = n.expr
        names: List[str] = []
        m = re.match(r"^\s*(\$\w+)\s*(?:,\s*(\$\w+))?\s*:=\s*(.*)$", expr, re.S)
        if m:
            names = [x for x in (m.group(1), m.group(2)) if x]
            expr = m.group(3)
        coll = self._pipeline(expr, dot, vars_)
        items: List[Tuple[Any, Any]]
        if isinstance(coll, dict):
            items = sorted(coll.items())
        elif isinstance(coll, (list, tuple)):
            items = list(enumerate(coll))
        elif isinstance(coll, int):
            items = [(i, i) for i in range(coll)]
        else:
            items = []
        if not items:
            self._exec(n.else_, dot, dict(vars_), out)
            return
        for k, v in items:
            vv = dict(vars_)
            if len(names) == 1:
                vv[names[0]] = v
            elif len(names) == 2:
                vv[names[0]] = k
                vv[names[1]] = v
            self._exec(n.body, v, vv, out)

    def _action(self, expr: str, dot, vars_):
        m = re.match(r"^\s*(\$\w+)\s*(:=|=)\s*(.*)$", expr, re.S)
        if m:
            vars_[m.group(1)] = self._pipeline(m.group(3), dot, vars_)
            return _NOOUT
        return self._pipeline(expr, dot, vars_)

    def _pipeline(self, expr: str, dot, vars_):
        return self._eval_tokens(_tokens(expr), dot, vars_)

    def _eval_tokens(self, toks: List[Tuple[str, str]], dot, vars_):
        # split on top-level pipes
        stages: List[List[Tuple[str, str]]] = [[]]
        depth = 0
        for t in toks:
            if t[0] == "lp":
                depth += 1
            elif t[0] == "rp":
                depth -= 1
            if t[0] == "pipe" and depth == 0:
                stages.append([])
            else:
                stages[-1].append(t)
        val = _NOVAL
        for st in stages:
            val = self._command(st, dot, vars_, val)
        return val

    def _command(self, toks, dot, vars_, piped):
        args: List[Any] = []
        i = 0
        fn_name = None
        if toks and toks[0][0] == "ident" and toks[0][1] not in ("true", "false", "nil"):
            fn_name = toks[0][1]
            i = 1
        while i < len(toks):
            kind, s = toks[i]
            if kind == "lp":
                depth, j = 1, i + 1
                while depth:
                    if toks[j][0] == "lp":
                        depth += 1
                    elif toks[j][0] == "rp":
                        depth -= 1
                    j += 1
                v = self._eval_tokens(toks[i + 1:j - 1], dot, vars_)
                for f in toks[j - 1][1].split(".")[1:]:
                    v = _field(v, f)
                args.append(v)
                i = j
                continue
            args.append(self._operand(kind, s, dot, vars_))
            i += 1
        if piped is not _NOVAL:
            args.append(piped)
        if fn_name is None:
            if len(args) != 1:
                raise TemplateError(f"cannot evaluate {toks}")
            return args[0]
        if fn_name == "include":
            return self._include(args[0], args[1] if len(args) > 1 else None)
        if fn_name == "tpl":
            t = Template()
            t.defines = self.defines
            t.add("_tpl", args[0])
            return t.render("_tpl", args[1])
        fn = FUNCS.get(fn_name)
        if fn is None:
            raise TemplateError(f"function {fn_name!r} not defined")
        return fn(*args)

    def _operand(self, kind, s, dot, vars_):
        if kind == "str":
            return _unquote(s)
        if kind == "raw":
            return s[1:-1]
        if kind == "num":
            return float(s) if "." in s else int(s)
        if kind == "ident":
            return {"true": True, "false": False, "nil": None}[s]
        if kind == "field":
            if s == ".":
                return dot
            v = dot
            for f in s.split(".")[1:]:
                v = _field(v, f)
            return v
        if kind == "var":
            parts = s.split(".")
            if parts[0] not in vars_:
                raise TemplateError(f"undefined variable {parts[0]}")
            v = vars_[parts[0]]
            for f in parts[1:]:
                v = _field(v, f)
            return v
        raise TemplateError(f"unexpected token {s!r}")

    def _include(self, name: str, arg) -> str:
        if name not in self.defines:
            raise TemplateError(f"template {name!r} not defined")
        out: List[str] = []
        self._exec(self.defines[name], arg, {"$": arg}, out)
        return "".join(out)


_NOOUT = object()
_NOVAL = object()


# ------------------------------------------------------------------------------------------
# Helm-like chart rendering
# ------------------------------------------------------------------------------------------
def deep_merge(base: Dict, over: Dict) -> Dict:
    out = dict(base)
    for k, v in (over or {}).items():
        if isinstance(v, dict) and isinstance(out.get(k), dict):
            out[k] = deep_merge(out[k], v)
        else:
            out[k] = v
    return out


def _load_chart(chart_dir: str) -> Tuple[Dict, Dict]:
    import os
    with open(os.path.join(chart_dir, "Chart.yaml")) as f:
        chart = yaml.safe_load(f)
    vals: Dict = {}
    if os.path.exists(os.path.join(chart_dir, "values.yaml")):
        with open(os.path.join(chart_dir, "values.yaml")) as f:
            vals = yaml.safe_load(f) or {}
    return chart, vals


def _condition_true(values: Dict, condition: str) -> bool:
    """Helm's dependency ``condition``: the first of its comma-separated value paths that
    resolves decides; none resolving keeps the dependency enabled."""
    for path in [c.strip() for c in (condition or "").split(",") if c.strip()]:
        cur: Any = values
        for part in path.split("."):
            if not isinstance(cur, dict) or part not in cur:
                cur = None
                break
            cur = cur[part]
        if isinstance(cur, bool):
            return cur
    return True


def kube_version(version: str) -> Dict[str, str]:
    """``.Capabilities.KubeVersion`` as Helm fills it: Version "v1.24.3", Major "1", Minor "24"; a
    provider build ("v1.24.3+eks") reports Minor "24+", as EKS / GKE clusters do."""
    plus = "+" in version
    v = version.lstrip("v").split("-")[0].split("+")[0].split(".")
    return {"Version": "v" + ".".join(v), "GitVersion": version, "Major": v[0],
            "Minor": (v[1] if len(v) > 1 else "0") + ("+" if plus else "")}


def render_chart(chart_dir: str, values: Optional[Dict] = None, release: str = "amd-gpu-operator",
                 namespace: str = "amd-gpu-operator", prefix: str = "", kube: str = "v1.29.0") -> Dict[str, str]:
    """Render every template of a chart and of its enabled dependencies vendored under
    ``charts/<name>/`` (the subchart sees its own values.yaml merged with the parent's
    ``<name>:`` section, as Helm does) for cluster version ``kube``; returns {template path:
    rendered text}."""
    import os
    chart, base = _load_chart(chart_dir)
    vals = deep_merge(base, values or {})
    dot = {"Values": vals, "Release": {"Name": release, "Namespace": namespace, "Service": "Helm"},
           "Chart": {"Name": chart["name"], "Version": chart["version"], "AppVersion": chart.get("appVersion", "")},
           "Capabilities": {"KubeVersion": kube_version(kube)}}
    t = Template()
    tdir = os.path.join(chart_dir, "templates")
    names = sorted(os.listdir(tdir))
    for n in names:
        with open(os.path.join(tdir, n)) as f:
            t.add(n, f.read())
    out = {prefix + "templates/" + n if prefix else n: t.render(n, dot)
           for n in names if not n.startswith("_") and n.endswith((".yaml", ".txt"))}
    for dep in chart.get("dependencies") or []:
        sub = os.path.join(chart_dir, "charts", dep["name"])
        if not os.path.isdir(sub) or not _condition_true(vals, dep.get("condition", "")):
            continue
        out.update(render_chart(sub, vals.get(dep.get("alias") or dep["name"]) or {}, release, namespace,
                                prefix=f"{prefix}charts/{dep['name']}/", kube=kube))
    return out


def chart_lock_digest(requested: List[Dict], locked: List[Dict]) -> str:
    """The ``digest`` Helm writes into Chart.lock: sha256 over the compact JSON of [the
    Chart.yaml dependencies, the locked ones], each encoded like Helm's chart.Dependency (name,
    version and condition omitted when empty, repository always)."""
    import hashlib
    import json

    def enc(d: Dict) -> Dict:
        out: Dict[str, Any] = {"name": d["name"]}
        if d.get("version"):
            out["version"] = d["version"]
        out["repository"] = d.get("repository", "")
        for k in ("condition", "tags", "enabled", "import-values", "alias"):
            if d.get(k):
                out[k] = d[k]
        return out
    data = json.dumps([[enc(d) for d in requested], [enc(d) for d in locked]], separators=(",", ":"))
    return "sha256:" + hashlib.sha256(data.encode()).hexdigest()


def render_objects(chart_dir: str, values: Optional[Dict] = None, **kw) -> List[Dict]:
    """Objects of every rendered template (subcharts included), plus the CRDs under the chart's
    and its enabled subcharts' ``crds/`` only with ``include_crds=True``."""
    import os
    include_crds = kw.pop("include_crds", False)
    out = []
    if include_crds:
        chart, base = _load_chart(chart_dir)
        vals = deep_merge(base, values or {})
        dirs = [chart_dir] + [os.path.join(chart_dir, "charts", d["name"]) for d in chart.get("dependencies") or []
                              if _condition_true(vals, d.get("condition", ""))]
        for d in dirs:
            for p in sorted(glob.glob(os.path.join(d, "crds", "*.yaml"))):
                with open(p) as f:
                    out += [doc for doc in yaml.safe_load_all(f) if doc]
    for name, text in render_chart(chart_dir, values, **kw).items():
        if not name.endswith(".yaml"):
            continue
        for doc in yaml.safe_load_all(text):
            if doc:
                out.append(doc)
    return out
