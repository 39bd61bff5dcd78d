"""A Go ``text/template`` subset interpreter with the Helm/Sprig functions the
machine-learning charts use (SURVEY §2.2 "Template functions used").

Supported syntax: ``{{ pipeline }}``, trim markers ``{{-`` / ``-}}``, comments
``{{/* */}}``, ``if / else if / else / end``, ``range`` (lists, maps in sorted-key order,
ints; ``$i, $v :=`` forms), ``with``, ``define`` / ``template`` / ``include``, variable
declaration ``$x := p`` and assignment ``$x = p`` (Go scoping: assignment updates the
innermost declaration, so ``$pv_index = add $pv_index 1`` inside a range carries over
iterations exactly like Helm), pipelines with ``|``, parenthesised sub-pipelines,
field chains on ``.``/``$``/variables, string/raw-string/number/bool/nil literals.

Functions: tpl include required fail default empty coalesce ternary quote squote
toYaml toJson indent nindent trim trimSuffix trimPrefix upper lower title replace
contains hasPrefix hasSuffix printf print println len list dict get set hasKey keys
first last join splitList toString int int64 float64 add sub mul div mod max min
add1 eq ne lt le gt ge and or not date now b64enc b64dec sha256sum trunc repeat
regexMatch semverCompare(true) lookup(empty).
"""
from __future__ import annotations

import base64
import datetime as _dt
import hashlib
import json
import re
from typing import Any, Callable, Dict, List, Optional, Tuple

import yaml


class TemplateError(Exception):
    pass


class _Required(TemplateError):
    pass


# ============================================================================ lexer
_ACTION = re.compile(
    r"\{\{(?P<cl>-\s)?\s*/\*.*?\*/\s*(?P<cr>\s-)?\}\}"      # comment (may contain '}}')
    r"|\{\{(?P<l>-\s)?(?P<body>.*?)(?P<r>\s-)?\}\}", re.S)


def _lex(src: str) -> List[Tuple[str, str]]:
    """Split into [("text", s) | ("action", s)] applying trim markers."""
    out: List[Tuple[str, str]] = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group("l") or m.group("cl"):  # {{- trims preceding whitespace
            text = text.rstrip(" \t\r\n")
        if out and out[-1][0] == "trimnext":
            out.pop()
            text = text.lstrip(" \t\r\n")
        if text:
            out.append(("text", text))
        if m.group("body") is not None:
            out.append(("action", m.group("body").strip()))
        if m.group("r") or m.group("cr"):
            out.append(("trimnext", ""))
        pos = m.end()
    text = src[pos:]
    if out and out[-1][0] == "trimnext":
        out.pop()
        text = text.lstrip(" \t\r\n")
    if text:
        out.append(("text", text))
    return [t for t in out if t[0] != "trimnext"]


# ============================================================================ expression tokens
_TOK = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>"(?:[^"\\]|\\.)*")
  | (?P<raw>`[^`]*`)
  | (?P<char>'(?:[^'\\]|\\.)')
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<pipe>\|)
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<comma>,)
  | (?P<num>-?\d+\.\d*(?:[eE][-+]?\d+)?|-?\d+[eE][-+]?\d+|-?0x[0-9a-fA-F]+|-?\d+)
  | (?P<var>\$[A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
  | (?P<field>(?:\.[A-Za-z0-9_]+)+|\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*(?:\.[A-Za-z0-9_]+)*)
""", re.X)


def _tokens(s: str):
    pos = 0
    out = []
    while pos < len(s):
        m = _TOK.match(s, pos)
        if not m:
            raise TemplateError(f"cannot tokenize {s[pos:]!r} in {{{{ {s} }}}}")
        pos = m.end()
        kind = m.lastgroup
        if kind == "ws":
            continue
        val = m.group(kind)
        if kind == "field" and out and out[-1][0] == "rp_done":
            pass
        out.append((kind, val))
    return out


# ============================================================================ AST
class Node:
    pass


class Text(Node):
    def __init__(self, s):
        self.s = s


class Output(Node):
    def __init__(self, pipe):
        self.pipe = pipe


class If(Node):
    def __init__(self, branches, else_body):
        self.branches = branches  # [(pipe, body)]
        self.else_body = else_body


class Range(Node):
    def __init__(self, keyvar, valvar, pipe, body, else_body):
        self.keyvar, self.valvar, self.pipe, self.body, self.else_body = (
            keyvar, valvar, pipe, body, else_body)


class With(Node):
    def __init__(self, pipe, body, else_body, var=None):
        self.pipe, self.body, self.else_body, self.var = pipe, body, else_body, var


class Define(Node):
    def __init__(self, name, body):
        self.name, self.body = name, body


class TemplateCall(Node):
    def __init__(self, name, pipe):
        self.name, self.pipe = name, pipe


class VarSet(Node):
    def __init__(self, name, pipe, declare):
        self.name, self.pipe, self.declare = name, pipe, declare


# a pipeline = (decl_vars, [command]); command = [arg]; arg = ("lit", v) | ("field", chain)
# | ("var", name, chain) | ("fn", name) | ("sub", pipeline) | ("subfield", pipeline, chain)


def _parse_pipeline(tokens, i=0, stop=None):
    cmds = []
    cur = []
    while i < len(tokens):
        kind, val = tokens[i]
        if stop and kind == stop:
            break
        if kind == "pipe":
            cmds.append(cur)
            cur = []
            i += 1
            continue
        if kind == "lp":
            sub, i = _parse_pipeline(tokens, i + 1, stop="rp")
            i += 1  # consume ')'
            # field access on a parenthesised pipeline: (x).Field
            if i < len(tokens) and tokens[i][0] == "field" and tokens[i][1] != ".":
                cur.append(("subfield", sub, tokens[i][1].split(".")[1:]))
                i += 1
            else:
                cur.append(("sub", sub))
            continue
        if kind == "str":
            cur.append(("lit", json.loads(val)))
        elif kind == "raw":
            cur.append(("lit", val[1:-1]))
        elif kind == "char":
            cur.append(("lit", ord(json.loads('"' + val[1:-1] + '"'))))
        elif kind == "num":
            v = val.lower()
            if v.startswith(("0x", "-0x")):
                cur.append(("lit", int(val, 16)))
            elif re.fullmatch(r"-?\d+", val):
                cur.append(("lit", int(val)))
            else:
                cur.append(("lit", float(val)))
        elif kind == "var":
            parts = val.split(".")
            cur.append(("var", parts[0], parts[1:]))
        elif kind == "field":
            chain = [] if val == "." else val.split(".")[1:]
            cur.append(("field", chain))
        elif kind == "ident":
            if val in ("true", "false"):
                cur.append(("lit", val == "true"))
            elif val == "nil":
                cur.append(("lit", None))
            else:
                cur.append(("fn", val))
        else:
            raise TemplateError(f"unexpected token {val!r}")
        i += 1
    cmds.append(cur)
    return cmds, i


def _parse_action_pipeline(s: str):
    toks = _tokens(s)
    # variable declaration / assignment:  $x := pipe  |  $x = pipe  |  $i, $v := pipe
    if len(toks) >= 2 and toks[0][0] == "var":
        if toks[1][0] in ("decl", "assign"):
            cmds, _ = _parse_pipeline(toks[2:])
            return ("set", toks[0][1], cmds, toks[1][0] == "decl")
        if toks[1][0] == "comma" and len(toks) >= 4 and toks[2][0] == "var" and toks[3][0] == "decl":
            cmds, _ = _parse_pipeline(toks[4:])
            return ("set2", toks[0][1], toks[2][1], cmds)
    cmds, _ = _parse_pipeline(toks)
    return ("pipe", cmds)


class _Parser:
    def __init__(self, items):
        self.items = items
        self.i = 0
        self.defines: Dict[str, List[Node]] = {}

    def parse(self, until=("end",)):
        body: List[Node] = []
        while self.i < len(self.items):
            kind, s = self.items[self.i]
            self.i += 1
            if kind == "text":
                body.append(Text(s))
                continue
            word = s.split(None, 1)[0] if s else ""
            rest = s[len(word):].strip()
            if word in ("end",):
                return body, "end", ""
            if word == "else":
                return body, "else", rest
            if word == "if":
                body.append(self._parse_if(rest))
            elif word == "range":
                body.append(self._parse_range(rest))
            elif word == "with":
                body.append(self._parse_with(rest))
            elif word in ("define", "block"):
                name = json.loads(rest.split()[0]) if rest.startswith('"') else rest.split()[0]
                inner, term, _ = self.parse()
                self.defines[name] = inner
                if word == "block":
                    pipe = rest[len(rest.split()[0]):].strip() or "."
                    body.append(TemplateCall(name, _parse_action_pipeline(pipe)[1]))
            elif word == "template":
                m = re.match(r'"([^"]*)"\s*(.*)', rest)
                if not m:
                    raise TemplateError(f"bad template call {s!r}")
                pipe = m.group(2).strip() or "."
                body.append(TemplateCall(m.group(1), _parse_action_pipeline(pipe)[1]))
            else:
                p = _parse_action_pipeline(s)
                if p[0] == "set":
                    body.append(VarSet(p[1], p[2], p[3]))
                elif p[0] == "set2":
                    raise TemplateError("two-variable declaration outside range")
                else:
                    body.append(Output(p[1]))
        return body, None, ""

    def _parse_if(self, cond):
        branches = []
        else_body = None
        body, term, rest = self.parse()
        branches.append((_parse_action_pipeline(cond)[1], body))
        while term == "else":
            if rest.startswith("if "):
                body, term, rest2 = self.parse()
                branches.append((_parse_action_pipeline(rest[3:])[1], body))
                rest = rest2
            else:
                else_body, term, _ = self.parse()
                break
        return If(branches, else_body)

    def _parse_range(self, spec):
        p = _parse_action_pipeline(spec)
        keyvar = valvar = None
        if p[0] == "set":
            valvar, pipe = p[1], p[2]
        elif p[0] == "set2":
            keyvar, valvar, pipe = p[1], p[2], p[3]
        else:
            pipe = p[1]
        body, term, _ = self.parse()
        else_body = None
        if term == "else":
            else_body, _, _ = self.parse()
        return Range(keyvar, valvar, pipe, body, else_body)

    def _parse_with(self, spec):
        p = _parse_action_pipeline(spec)
        var = None
        if p[0] == "set":
            var, pipe = p[1], p[2]
        else:
            pipe = p[1]
        body, term, _ = self.parse()
        else_body = None
        if term == "else":
            else_body, _, _ = self.parse()
        return With(pipe, body, else_body, var)


# ============================================================================ values
def truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, list, dict, tuple)):
        return len(v) > 0
    return True


def to_str(v) -> str:
    """Go %v formatting of YAML-decoded values (Helm renders nil as empty)."""
    if v is None:
        return ""
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        if v == int(v) and abs(v) < 1e21:
            return str(int(v)) if abs(v) < 1e6 else f"{v:g}".replace("e+0", "e+")
        return repr(v)
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{to_str(v[k])}" for k in sorted(v)) + "]"
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(to_str(x) for x in v) + "]"
    return str(v)


def _go_date(layout: str, t: _dt.datetime) -> str:
    repl = [("2006", "%Y"), ("01", "%m"), ("02", "%d"), ("15", "%H"), ("04", "%M"),
            ("05", "%S"), ("Jan", "%b"), ("Mon", "%a"), ("MST", "%Z"), ("-0700", "%z")]
    out = ""
    i = 0
    while i < len(layout):
        for g, p in repl:
            if layout.startswith(g, i):
                out += t.strftime(p)
                i += len(g)
                break
        else:
            out += layout[i]
            i += 1
    return out


def _num(v):
    if isinstance(v, bool):
        return int(v)
    if isinstance(v, (int, float)):
        return v
    if v is None or v == "":
        return 0
    try:
        return int(v)
    except (TypeError, ValueError):
        return float(v)


def _to_int(v):
    try:
        return int(float(_num(v)))
    except (TypeError, ValueError):
        return 0


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + line for line in to_str(s).split("\n"))


def _to_yaml(v):
    if v is None:
        return "null"
    return yaml.safe_dump(v, default_flow_style=False, sort_keys=True).rstrip("\n")


def _printf(fmt, *args):
    # translate Go verbs to Python %-format
    conv = re.sub(r"%v|%s", "%s", fmt)
    conv = re.sub(r"%q", '"%s"', conv)
    conv = re.sub(r"%d", "%d", conv)
    vals = tuple(to_str(a) if re.search(r"%s", conv) and not isinstance(a, (int, float)) else a
                 for a in args)
    try:
        return conv % vals
    except TypeError:
        return conv % tuple(to_str(a) for a in args)


# ============================================================================ evaluation
class _Scope:
    def __init__(self, parent=None):
        self.vars: Dict[str, Any] = {}
        self.parent = parent

    def get(self, name):
        s = self
        while s is not None:
            if name in s.vars:
                return s.vars[name]
            s = s.parent
        raise TemplateError(f"undefined variable {name}")

    def declare(self, name, v):
        self.vars[name] = v

    def assign(self, name, v):
        s = self
        while s is not None:
            if name in s.vars:
                s.vars[name] = v
                return
            s = s.parent
        raise TemplateError(f"assignment to undeclared variable {name}")


def _field(obj, chain, strict=False):
    for k in chain:
        if obj is None:
            return None
        if isinstance(obj, dict):
            obj = obj.get(k)
        else:
            obj = getattr(obj, k, None)
    return obj


class Engine:
    """Renders templates of one chart (shares ``define``s across files)."""

    def __init__(self):
        self.defines: Dict[str, List[Node]] = {}
        self.funcs: Dict[str, Callable] = self._builtin_funcs()
        self.root: Any = None

    # ---------------------------------------------------------------- API
    def parse(self, src: str) -> List[Node]:
        p = _Parser(_lex(src))
        body, term, _ = p.parse()
        if term is not None:
            raise TemplateError(f"unexpected {{{{{term}}}}}")
        self.defines.update(p.defines)
        return body

    def render(self, src_or_nodes, dot, root=None) -> str:
        nodes = self.parse(src_or_nodes) if isinstance(src_or_nodes, str) else src_or_nodes
        self.root = root if root is not None else dot
        scope = _Scope()
        scope.declare("$", self.root)
        out: List[str] = []
        self._exec(nodes, dot, scope, out)
        return "".join(out)

    # ---------------------------------------------------------------- exec
    def _exec(self, nodes, dot, scope, out):
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.s)
            elif isinstance(n, Output):
                out.append(to_str(self._pipe(n.pipe, dot, scope)))
            elif isinstance(n, VarSet):
                v = self._pipe(n.pipe, dot, scope)
                if n.declare:
                    scope.declare(n.name, v)
                else:
                    scope.assign(n.name, v)
            elif isinstance(n, If):
                for cond, body in n.branches:
                    if truthy(self._pipe(cond, dot, scope)):
                        self._exec(body, dot, _Scope(scope), out)
                        break
                else:
                    if n.else_body is not None:
                        self._exec(n.else_body, dot, _Scope(scope), out)
            elif isinstance(n, With):
                v = self._pipe(n.pipe, dot, scope)
                if truthy(v):
                    s = _Scope(scope)
                    if n.var:
                        s.declare(n.var, v)
                    self._exec(n.body, v, s, out)
                elif n.else_body is not None:
                    self._exec(n.else_body, dot, _Scope(scope), out)
            elif isinstance(n, Range):
                v = self._pipe(n.pipe, dot, scope)
                items: List[Tuple[Any, Any]]
                if isinstance(v, dict):
                    items = [(k, v[k]) for k in sorted(v)]
                elif isinstance(v, (list, tuple)):
                    items = list(enumerate(v))
                elif isinstance(v, int) and not isinstance(v, bool):
                    items = [(i, i) for i in range(v)]
                elif v is None:
                    items = []
                else:
                    raise TemplateError(f"range over {type(v).__name__}")
                if not items:
                    if n.else_body is not None:
                        self._exec(n.else_body, dot, _Scope(scope), out)
                    continue
                for k, item in items:
                    s = _Scope(scope)
                    if n.keyvar:
                        s.declare(n.keyvar, k)
                    if n.valvar:
                        s.declare(n.valvar, item)
                    self._exec(n.body, item, s, out)
            elif isinstance(n, TemplateCall):
                arg = self._pipe(n.pipe, dot, scope)
                out.append(self.include(n.name, arg))
            elif isinstance(n, Define):
                self.defines[n.name] = n.body

    def include(self, name, dot):
        if name not in self.defines:
            raise TemplateError(f"template {name!r} not defined")
        s = _Scope()
        s.declare("$", dot)  # Go: `$` inside a template is the data it was invoked with
        out: List[str] = []
        self._exec(self.defines[name], dot, s, out)
        return "".join(out)

    def _pipe(self, cmds, dot, scope):
        val = _NOARG = object()
        for cmd in cmds:
            val = self._cmd(cmd, dot, scope, None if val is _NOARG else val, val is not _NOARG)
        return None if val is _NOARG else val

    def _arg(self, a, dot, scope):
        kind = a[0]
        if kind == "lit":
            return a[1]
        if kind == "field":
            return _field(dot, a[1])
        if kind == "var":
            return _field(scope.get(a[1]), a[2])
        if kind == "sub":
            return self._pipe(a[1], dot, scope)
        if kind == "subfield":
            return _field(self._pipe(a[1], dot, scope), a[2])
        if kind == "fn":
            return self._call(a[1], [], dot, scope)
        raise TemplateError(f"bad arg {a}")

    def _cmd(self, cmd, dot, scope, piped, has_piped):
        if not cmd:
            raise TemplateError("empty command")
        head = cmd[0]
        if head[0] == "fn":
            args = [self._arg(a, dot, scope) for a in cmd[1:]]
            if has_piped:
                args.append(piped)
            return self._call(head[1], args, dot, scope)
        if len(cmd) > 1:
            raise TemplateError(f"can't give argument to non-function {head}")
        return self._arg(head, dot, scope)

    def _call(self, name, args, dot, scope):
        if name not in self.funcs:
            raise TemplateError(f'function "{name}" not defined')
        return self.funcs[name](*args)

    # ---------------------------------------------------------------- funcs
    def _tpl(self, s, ctx):
        sub = Engine()
        sub.defines = self.defines
        sub.funcs = self.funcs
        return sub.render(to_str(s), ctx, root=ctx)

    def _builtin_funcs(self) -> Dict[str, Callable]:
        def required(msg, v=None):
            if v is None or v == "":
                raise _Required(msg)
            return v

        def fail(msg):
            raise TemplateError(msg)

        def default(d, v=None):
            return v if truthy(v) else d

        def date(layout, t=None):
            if t is None:
                t = _dt.datetime.now()
            if isinstance(t, str):
                t = _dt.datetime.fromisoformat(t)
            return _go_date(layout, t)

        def dict_(*kv):
            return {to_str(kv[i]): kv[i + 1] for i in range(0, len(kv) - 1, 2)}

        def div(a, b):
            a, b = _num(a), _num(b)
            return a // b if isinstance(a, int) and isinstance(b, int) else a / b

        def eq(a, *bs):
            return any(a == b for b in bs)

        def and_(*xs):
            v = True
            for x in xs:
                v = x
                if not truthy(x):
                    return x
            return v

        def or_(*xs):
            v = False
            for x in xs:
                v = x
                if truthy(x):
                    return x
            return v

        def index(obj, *keys):
            for k in keys:
                if obj is None:
                    return None
                if isinstance(obj, (list, tuple)):
                    obj = obj[int(k)] if int(k) < len(obj) else None
                elif isinstance(obj, dict):
                    obj = obj.get(k)
                else:
                    obj = getattr(obj, str(k), None)
            return obj

        return {
            "index": index,
            "tpl": self._tpl,
            "include": lambda name, d=None: self.include(name, d),
            "required": required,
            "fail": fail,
            "default": default,
            "empty": lambda v=None: not truthy(v),
            "coalesce": lambda *xs: next((x for x in xs if truthy(x)), None),
            "ternary": lambda a, b, c: a if truthy(c) else b,
            "quote": lambda *xs: " ".join('"' + to_str(x).replace('"', '\\"') + '"' for x in xs),
            "squote": lambda *xs: " ".join("'" + to_str(x) + "'" for x in xs),
            "toYaml": _to_yaml,
            "toJson": lambda v: json.dumps(v, sort_keys=True),
            "fromYaml": lambda s: yaml.safe_load(to_str(s)) or {},
            "indent": _indent,
            "nindent": lambda n, s: "\n" + _indent(n, s),
            "trim": lambda s: to_str(s).strip(),
            "trimSuffix": lambda suf, s: to_str(s)[: -len(suf)] if to_str(s).endswith(suf) and suf else to_str(s),
            "trimPrefix": lambda pre, s: to_str(s)[len(pre):] if to_str(s).startswith(pre) else to_str(s),
            "upper": lambda s: to_str(s).upper(),
            "lower": lambda s: to_str(s).lower(),
            "title": lambda s: to_str(s).title(),
            "replace": lambda old, new, s: to_str(s).replace(old, new),
            "contains": lambda sub, s: sub in to_str(s),
            "hasPrefix": lambda pre, s: to_str(s).startswith(pre),
            "hasSuffix": lambda suf, s: to_str(s).endswith(suf),
            "printf": _printf,
            "print": lambda *xs: "".join(to_str(x) for x in xs),
            "println": lambda *xs: " ".join(to_str(x) for x in xs) + "\n",
            "len": lambda v: len(v) if v is not None else 0,
            "list": lambda *xs: list(xs),
            "dict": dict_,
            "get": lambda d, k: (d or {}).get(k, ""),
            "set": lambda d, k, v: (d.__setitem__(k, v), d)[1],
            "hasKey": lambda d, k: k in (d or {}),
            "keys": lambda *ds: sorted(k for d in ds for k in (d or {})),
            "first": lambda v: v[0] if v else None,
            "last": lambda v: v[-1] if v else None,
            "join": lambda sep, v: sep.join(to_str(x) for x in (v or [])),
            "splitList": lambda sep, s: to_str(s).split(sep),
            "toString": to_str,
            "int": _to_int,
            "int64": _to_int,
            "float64": lambda v: float(_num(v)),
            "add": lambda *xs: sum(_num(x) for x in xs),
            "add1": lambda x: _num(x) + 1,
            "sub": lambda a, b: _num(a) - _num(b),
            "mul": lambda *xs: __import__("math").prod(_num(x) for x in xs),
            "div": div,
            "mod": lambda a, b: _num(a) % _num(b),
            "max": lambda *xs: max(_num(x) for x in xs),
            "min": lambda *xs: min(_num(x) for x in xs),
            "eq": eq,
            "ne": lambda a, b: a != b,
            "lt": lambda a, b: _num(a) < _num(b),
            "le": lambda a, b: _num(a) <= _num(b),
            "gt": lambda a, b: _num(a) > _num(b),
            "ge": lambda a, b: _num(a) >= _num(b),
            "and": and_,
            "or": or_,
            "not": lambda v: not truthy(v),
            "date": date,
            "now": lambda: _dt.datetime.now(),
            "b64enc": lambda s: base64.b64encode(to_str(s).encode()).decode(),
            "b64dec": lambda s: base64.b64decode(to_str(s)).decode(),
            "sha256sum": lambda s: hashlib.sha256(to_str(s).encode()).hexdigest(),
            "trunc": lambda n, s: to_str(s)[: int(n)] if int(n) >= 0 else to_str(s)[int(n):],
            "repeat": lambda n, s: to_str(s) * int(n),
            "regexMatch": lambda rx, s: re.search(rx, to_str(s)) is not None,
            "semverCompare": lambda c, v: True,
            "lookup": lambda *a: {},
        }


def render_string(src: str, dot: Any, root: Any = None) -> str:
    return Engine().render(src, dot, root)
