"""A Go `text/template` interpreter (with the sprig functions model templates use).

Model YAMLs in the LocalAI gallery carry prompt templates in Go template syntax
(pkg/templates/cache.go:79 parses them with text/template + sprig). This is an independent
implementation of that language subset in Python:

  text, {{ action }}, trim markers {{- -}}, comments {{/* */}}
  pipelines: .Field.Path, $var, $, literals ("s", `raw`, 'c', 1, 1.5, true, false, nil),
             function calls, `|` chaining, parenthesised sub-pipelines, method-less field access
  actions:   if / else if / else / end, range (with `$i, $v := range`), with, define,
             template, block, break, continue, variable declare/assign (:= / =)
  builtins:  and or not len index slice print printf println eq ne lt le gt ge html js urlquery call
  sprig:     toJson toPrettyJson fromJson trim trimSuffix trimPrefix trimAll upper lower title
             contains hasPrefix hasSuffix replace join split splitList default empty coalesce
             list dict get set hasKey keys add sub mul div mod max min quote squote indent
             nindent repeat toString atoi int float64 regexMatch regexReplaceAll regexFind
             substr trunc first last uniq sortAlpha ternary now date b64enc b64dec
"""
from __future__ import annotations

import base64
import datetime
import html as _html
import json
import re
import urllib.parse
from dataclasses import dataclass, field


class TemplateError(Exception):
    pass


# ------------------------------------------------------------------------------------------------
# lexer: split into text / action chunks, honouring trim markers

_ACTION = re.compile(r"\{\{(-\s)?(.*?)(\s-)?\}\}", re.S)


def _split(src: str):
    out = []
    pos = 0
    for m in _ACTION.finditer(src):
        text = src[pos:m.start()]
        if m.group(1):
            text = text.rstrip(" \t\r\n")
        out.append(("text", text))
        body = m.group(2)
        out.append(("action", body.strip(), bool(m.group(3))))
        pos = m.end()
    out.append(("text", src[pos:]))
    # apply right-trim: an action with "-}}" trims leading whitespace of the next text
    res = []
    trim_next = False
    for it in out:
        if it[0] == "text":
            t = it[1]
            if trim_next:
                t = t.lstrip(" \t\r\n")
            res.append(("text", t))
            trim_next = False
        else:
            res.append(("action", it[1]))
            trim_next = it[2]
    return res


_TOKEN = re.compile(r"""
    (?P<ws>\s+)
  | (?P<str>"(?:\\.|[^"\\])*")
  | (?P<raw>`[^`]*`)
  | (?P<chr>'(?:\\.|[^'\\])')
  | (?P<num>-?\d+\.\d*|-?\d+)
  | (?P<decl>:=)
  | (?P<assign>=)
  | (?P<pipe>\|)
  | (?P<lp>\()
  | (?P<rp>\))
  | (?P<comma>,)
  | (?P<var>\$[A-Za-z0-9_]*)
  | (?P<field>(?:\.[A-Za-z0-9_]+)+|\.)
  | (?P<ident>[A-Za-z_][A-Za-z0-9_]*)
""", re.X)


def _tokens(s: str):
    toks = []
    pos = 0
    while pos < len(s):
        m = _TOKEN.match(s, pos)
        if not m:
            raise TemplateError(f"bad token at {s[pos:pos + 20]!r}")
        kind = m.lastgroup
        val = m.group(kind)
        pos = m.end()
        if kind == "ws":
            continue
        # field access chained onto a variable / paren: $x.Foo  or (..).Foo
        if kind == "field" and toks and toks[-1][0] in ("var", "rp", "fieldof") and not s[m.start() - 1].isspace():
            toks.append(("fieldof", val))
            continue
        toks.append((kind, val))
    return toks


# ------------------------------------------------------------------------------------------------
# AST


@dataclass
class Node:
    pass


@dataclass
class Text(Node):
    text: str


@dataclass
class Action(Node):
    pipe: object  # Pipeline


@dataclass
class If(Node):
    branches: list  # [(pipe, [nodes])]
    else_: list | None


@dataclass
class Range(Node):
    pipe: object
    body: list
    else_: list | None


@dataclass
class With(Node):
    branches: list
    else_: list | None


@dataclass
class TemplateCall(Node):
    name: str
    pipe: object | None


@dataclass
class Break(Node):
    pass


@dataclass
class Continue(Node):
    pass


@dataclass
class Pipeline:
    decl: list  # variable names
    is_assign: bool
    cmds: list  # [[args]]


class _Brk(Exception):
    pass


class _Cont(Exception):
    pass


# ------------------------------------------------------------------------------------------------
# parser


class _Parser:
    def __init__(self, chunks, defines):
        self.chunks = chunks
        self.i = 0
        self.defines = defines

    def parse_list(self, stop=("end",)):
        nodes = []
        while self.i < len(self.chunks):
            ch = self.chunks[self.i]
            if ch[0] == "text":
                if ch[1]:
                    nodes.append(Text(ch[1]))
                self.i += 1
                continue
            body = ch[1]
            if body.startswith("/*"):
                self.i += 1
                continue
            word = body.split(None, 1)[0] if body else ""
            if word in stop or (word == "else" and "else" in stop):
                return nodes, body
            self.i += 1
            nodes.append(self.parse_action(body))
        return nodes, None

    def parse_action(self, body):
        word, _, rest = body.partition(" ")
        rest = rest.strip()
        if word == "if":
            return self._parse_cond(If, rest)
        if word == "with":
            return self._parse_cond(With, rest)
        if word == "range":
            pipe = self.parse_pipe(rest)
            body_nodes, end = self.parse_list(("end", "else"))
            else_ = None
            if end and end.startswith("else"):
                self.i += 1
                else_, end = self.parse_list(("end",))
            self._expect_end(end)
            return Range(pipe, body_nodes, else_)
        if word in ("define", "block"):
            toks = _tokens(rest)
            name = json.loads(toks[0][1]) if toks[0][0] == "str" else toks[0][1].strip("`")
            body_nodes, end = self.parse_list(("end",))
            self._expect_end(end)
            self.defines[name] = body_nodes
            if word == "block":
                pipe = self.parse_pipe(rest[len(toks[0][1]):]) if len(toks) > 1 else None
                return TemplateCall(name, pipe)
            return Text("")
        if word == "template":
            toks = _tokens(rest)
            name = json.loads(toks[0][1]) if toks[0][0] == "str" else toks[0][1].strip("`")
            after = rest[rest.index(toks[0][1]) + len(toks[0][1]):].strip()
            return TemplateCall(name, self.parse_pipe(after) if after else None)
        if word == "break":
            return Break()
        if word == "continue":
            return Continue()
        return Action(self.parse_pipe(body))

    def _expect_end(self, end):
        if end is None or not end.startswith("end"):
            raise TemplateError("missing {{end}}")
        self.i += 1

    def _parse_cond(self, cls, rest):
        branches = [(self.parse_pipe(rest), None)]
        nodes, end = self.parse_list(("end", "else"))
        branches[0] = (branches[0][0], nodes)
        else_ = None
        while end is not None and end.startswith("else"):
            self.i += 1
            tail = end[4:].strip()
            if tail.startswith("if ") or tail.startswith("with "):
                kw, _, cond = tail.partition(" ")
                nodes, end = self.parse_list(("end", "else"))
                branches.append((self.parse_pipe(cond), nodes))
                continue
            else_, end = self.parse_list(("end",))
            break
        self._expect_end(end)
        return cls(branches, else_)

    def parse_pipe(self, s):
        toks = _tokens(s)
        decl, is_assign = [], False
        # variable declaration:  $x := ...   |  $i, $v := ...
        j = 0
        names = []
        while j < len(toks) and toks[j][0] == "var":
            names.append(toks[j][1])
            if j + 1 < len(toks) and toks[j + 1][0] == "comma":
                j += 2
                continue
            j += 1
            break
        if names and j < len(toks) and toks[j][0] in ("decl", "assign"):
            decl = names
            is_assign = toks[j][0] == "assign"
            toks = toks[j + 1:]
        cmds = [[]]
        stack = []
        k = 0
        while k < len(toks):
            kind, val = toks[k]
            if kind == "pipe" and not stack:
                cmds.append([])
            elif kind == "lp":
                depth = 1
                m = k + 1
                while m < len(toks) and depth:
                    if toks[m][0] == "lp":
                        depth += 1
                    elif toks[m][0] == "rp":
                        depth -= 1
                    m += 1
                inner = toks[k + 1:m - 1]
                sub = self._pipe_from_tokens(inner)
                arg = ("pipe", sub)
                # trailing .Field after ')'
                while m < len(toks) and toks[m][0] == "fieldof":
                    arg = ("chain", arg, toks[m][1])
                    m += 1
                cmds[-1].append(arg)
                k = m
                continue
            elif kind == "fieldof":
                prev = cmds[-1].pop()
                cmds[-1].append(("chain", prev, val))
            else:
                cmds[-1].append((kind, val))
            k += 1
        return Pipeline(decl, is_assign, cmds)

    def _pipe_from_tokens(self, toks):
        # re-serialise is error prone; build directly
        cmds = [[]]
        k = 0
        while k < len(toks):
            kind, val = toks[k]
            if kind == "pipe":
                cmds.append([])
            elif kind == "lp":
                depth = 1
                m = k + 1
                while m < len(toks) and depth:
                    depth += 1 if toks[m][0] == "lp" else (-1 if toks[m][0] == "rp" else 0)
                    m += 1
                arg = ("pipe", self._pipe_from_tokens(toks[k + 1:m - 1]))
                while m < len(toks) and toks[m][0] == "fieldof":
                    arg = ("chain", arg, toks[m][1])
                    m += 1
                cmds[-1].append(arg)
                k = m
                continue
            elif kind == "fieldof":
                prev = cmds[-1].pop()
                cmds[-1].append(("chain", prev, val))
            else:
                cmds[-1].append((kind, val))
            k += 1
        return Pipeline([], False, cmds)


# ------------------------------------------------------------------------------------------------
# evaluation helpers


def truthy(v) -> bool:
    if v is None or v is False:
        return False
    if isinstance(v, (int, float)) and not isinstance(v, bool):
        return v != 0
    if isinstance(v, (str, bytes, list, tuple, dict, set)):
        return len(v) > 0
    return True


def _field(obj, name):
    if obj is None:
        return None
    if isinstance(obj, dict):
        if name in obj:
            return obj[name]
        # Go structs are usually exposed as dicts with Go field names; fall back to lower-snake
        alt = re.sub(r"(?<!^)(?=[A-Z])", "_", name).lower()
        return obj.get(alt)
    return getattr(obj, name, None)


def _go_str(v) -> str:
    if v is None:
        return "<no value>"
    if isinstance(v, bool):
        return "true" if v else "false"
    if isinstance(v, float):
        return repr(v) if v != int(v) else str(int(v)) if abs(v) < 1e21 else repr(v)
    if isinstance(v, (list, tuple)):
        return "[" + " ".join(_go_str(x) for x in v) + "]"
    if isinstance(v, dict):
        return "map[" + " ".join(f"{k}:{_go_str(x)}" for k, x in sorted(v.items(), key=lambda kv: str(kv[0]))) + "]"
    return str(v)


def _printf(fmt, *args):
    # translate Go verbs to Python %-format
    out = []
    ai = 0
    i = 0
    while i < len(fmt):
        c = fmt[i]
        if c != "%":
            out.append(c)
            i += 1
            continue
        j = i + 1
        while j < len(fmt) and fmt[j] in "+-# 0123456789.":
            j += 1
        if j >= len(fmt):
            out.append(fmt[i:])
            break
        verb = fmt[j]
        spec = fmt[i + 1:j]
        if verb == "%":
            out.append("%")
        else:
            a = args[ai] if ai < len(args) else None
            ai += 1
            if verb in "vs":
                out.append(("%" + spec + "s") % _go_str(a))
            elif verb == "q":
                out.append(json.dumps(_go_str(a)))
            elif verb in "dxXob":
                out.append(("%" + spec + verb.replace("b", "d")) % int(a))
            elif verb in "feEgG":
                out.append(("%" + spec + verb) % float(a))
            elif verb == "t":
                out.append("true" if a else "false")
            elif verb == "c":
                out.append(chr(int(a)))
            else:
                out.append(_go_str(a))
        i = j + 1
    return "".join(out)


def _cmp(a, b):
    if isinstance(a, (int, float)) and isinstance(b, (int, float)):
        return (a > b) - (a < b)
    a, b = str(a), str(b)
    return (a > b) - (a < b)


def _to_json(v, indent=None):
    def conv(x):
        if hasattr(x, "to_dict"):
            return x.to_dict()
        if hasattr(x, "__dict__") and not isinstance(x, type):
            return {k: v for k, v in vars(x).items() if not k.startswith("_")}
        return str(x)
    return json.dumps(v, default=conv, ensure_ascii=False, indent=indent, separators=(",", ":") if indent is None else None)


def _indent(n, s):
    pad = " " * int(n)
    return "\n".join(pad + line for line in str(s).split("\n"))


def _default(d, *v):
    val = v[0] if v else None
    return val if truthy(val) else d


BUILTINS = {
    "and": None, "or": None,  # short-circuit, handled in eval
    "not": lambda x: not truthy(x),
    "len": lambda x: len(x) if x is not None else 0,
    "index": lambda x, *ks: _index(x, ks),
    "slice": lambda x, *a: x[int(a[0]) if a else 0:int(a[1]) if len(a) > 1 else None],
    "print": lambda *a: "".join(_go_str(x) for x in a),
    "println": lambda *a: " ".join(_go_str(x) for x in a) + "\n",
    "printf": _printf,
    "eq": lambda a, *bs: any(a == b for b in bs),
    "ne": lambda a, b: a != b,
    "lt": lambda a, b: _cmp(a, b) < 0,
    "le": lambda a, b: _cmp(a, b) <= 0,
    "gt": lambda a, b: _cmp(a, b) > 0,
    "ge": lambda a, b: _cmp(a, b) >= 0,
    "html": lambda *a: _html.escape("".join(_go_str(x) for x in a)),
    "js": lambda *a: json.dumps("".join(_go_str(x) for x in a))[1:-1],
    "urlquery": lambda *a: urllib.parse.quote_plus("".join(_go_str(x) for x in a)),
    "call": lambda f, *a: f(*a),
    # sprig subset
    "toJson": _to_json, "mustToJson": _to_json,
    "toPrettyJson": lambda v: _to_json(v, 2), "fromJson": lambda s: json.loads(s) if s else None,
    "toString": _go_str,
    "trim": lambda s: str(s).strip(), "trimAll": lambda c, s: str(s).strip(c),
    "trimSuffix": lambda suf, s: str(s)[:-len(suf)] if suf and str(s).endswith(suf) else str(s),
    "trimPrefix": lambda pre, s: str(s)[len(pre):] if pre and str(s).startswith(pre) else str(s),
    "upper": lambda s: str(s).upper(), "lower": lambda s: str(s).lower(), "title": lambda s: str(s).title(),
    "contains": lambda sub, s: str(sub) in str(s),
    "hasPrefix": lambda pre, s: str(s).startswith(str(pre)),
    "hasSuffix": lambda suf, s: str(s).endswith(str(suf)),
    "replace": lambda old, new, s: str(s).replace(str(old), str(new)),
    "join": lambda sep, xs: str(sep).join(_go_str(x) for x in (xs or [])),
    "split": lambda sep, s: {f"_{i}": p for i, p in enumerate(str(s).split(sep))},
    "splitList": lambda sep, s: str(s).split(sep),
    "default": _default,
    "empty": lambda x: not truthy(x),
    "coalesce": lambda *a: next((x for x in a if truthy(x)), None),
    "list": lambda *a: list(a),
    "dict": lambda *a: {str(a[i]): a[i + 1] if i + 1 < len(a) else None for i in range(0, len(a), 2)},
    "get": lambda d, k: (d or {}).get(k, ""),
    "set": lambda d, k, v: (d.__setitem__(k, v), d)[1],
    "hasKey": lambda d, k: k in (d or {}),
    "keys": lambda *ds: [k for d in ds for k in (d or {})],
    "add": lambda *a: sum(_num(x) for x in a), "add1": lambda x: _num(x) + 1,
    "sub": lambda a, b: _num(a) - _num(b), "mul": lambda *a: _prod(a),
    "div": lambda a, b: _num(a) // _num(b) if isinstance(_num(a), int) and isinstance(_num(b), int) else _num(a) / _num(b),
    "mod": lambda a, b: _num(a) % _num(b),
    "max": lambda *a: max(_num(x) for x in a), "min": lambda *a: min(_num(x) for x in a),
    "quote": lambda *a: " ".join(json.dumps(_go_str(x)) for x in a),
    "squote": lambda *a: " ".join("'" + _go_str(x) + "'" for x in a),
    "indent": _indent, "nindent": lambda n, s: "\n" + _indent(n, s),
    "repeat": lambda n, s: str(s) * int(n),
    "atoi": lambda s: int(s), "int": lambda s: int(float(s)) if s not in (None, "") else 0,
    "int64": lambda s: int(float(s)) if s not in (None, "") else 0, "float64": lambda s: float(s),
    "regexMatch": lambda rx, s: re.search(rx, str(s)) is not None,
    "regexReplaceAll": lambda rx, s, repl: re.sub(rx, re.sub(r"\$\{?(\d+)\}?", r"\\\1", repl), str(s)),
    "regexFind": lambda rx, s: (m.group(0) if (m := re.search(rx, str(s))) else ""),
    "substr": lambda a, b, s: str(s)[int(a):int(b)] if int(b) >= 0 else str(s)[int(a):],
    "trunc": lambda n, s: str(s)[:int(n)] if int(n) >= 0 else str(s)[int(n):],
    "first": lambda xs: xs[0] if xs else None, "last": lambda xs: xs[-1] if xs else None,
    "uniq": lambda xs: list(dict.fromkeys(xs or [])), "sortAlpha": lambda xs: sorted(str(x) for x in (xs or [])),
    "ternary": lambda a, b, c: a if truthy(c) else b,
    "now": lambda: datetime.datetime.now(),
    "date": lambda fmt, t: (t or datetime.datetime.now()).strftime(_go_date_fmt(fmt)),
    "b64enc": lambda s: base64.b64encode(str(s).encode()).decode(),
    "b64dec": lambda s: base64.b64decode(str(s)).decode(errors="replace"),
}


def _go_date_fmt(fmt):
    for go, py in (("2006", "%Y"), ("01", "%m"), ("02", "%d"), ("15", "%H"), ("04", "%M"), ("05", "%S"),
                   ("Jan", "%b"), ("Mon", "%a")):
        fmt = fmt.replace(go, py)
    return fmt


def _num(x):
    if isinstance(x, (int, float)):
        return x
    try:
        return int(x)
    except (TypeError, ValueError):
        return float(x)


def _prod(a):
    r = 1
    for x in a:
        r *= _num(x)
    return r


def _index(x, ks):
    for k in ks:
        if x is None:
            return None
        if isinstance(x, dict):
            x = x.get(k)
        else:
            try:
                x = x[int(k)]
            except (IndexError, TypeError, ValueError):
                raise TemplateError(f"index out of range: {k}")
    return x


# ------------------------------------------------------------------------------------------------


class Template:
    def __init__(self, src: str, name: str = "tpl", funcs: dict | None = None):
        self.name = name
        self.defines: dict[str, list] = {}
        self.funcs = dict(BUILTINS)
        if funcs:
            self.funcs.update(funcs)
        p = _Parser(_split(src), self.defines)
        self.root, end = p.parse_list(())
        if end is not None:
            raise TemplateError(f"unexpected {{{{{end}}}}}")

    def render(self, data) -> str:
        out: list[str] = []
        self._exec(self.root, data, [{"$": data}], out)
        return "".join(out)

    # ------------------------------------------------------------------
    def _lookup_var(self, name, scopes):
        for s in reversed(scopes):
            if name in s:
                return s[name]
        raise TemplateError(f"undefined variable {name}")

    def _set_var(self, name, val, scopes, declare):
        if declare:
            scopes[-1][name] = val
            return
        for s in reversed(scopes):
            if name in s:
                s[name] = val
                return
        raise TemplateError(f"undefined variable {name}")

    def _arg(self, a, dot, scopes):
        kind = a[0]
        if kind == "field":
            if a[1] == ".":
                return dot
            v = dot
            for part in a[1].split(".")[1:]:
                v = _field(v, part)
            return v
        if kind == "var":
            return self._lookup_var(a[1] or "$", scopes)
        if kind == "chain":
            v = self._arg(a[1], dot, scopes)
            for part in a[2].split(".")[1:]:
                v = _field(v, part)
            return v
        if kind == "str":
            return json.loads(a[1])
        if kind == "raw":
            return a[1][1:-1]
        if kind == "chr":
            return ord(json.loads('"' + a[1][1:-1] + '"'))
        if kind == "num":
            return float(a[1]) if "." in a[1] else int(a[1])
        if kind == "pipe":
            return self._pipe(a[1], dot, scopes)
        if kind == "ident":
            if a[1] in ("true", "false"):
                return a[1] == "true"
            if a[1] == "nil":
                return None
            return self._call(a[1], [], dot, scopes)
        raise TemplateError(f"bad argument {a}")

    def _call(self, name, args, dot, scopes, prev=None, has_prev=False):
        if name in ("and", "or"):
            vals = list(args) + ([prev] if has_prev else [])
            res = None
            for i, x in enumerate(vals):
                v = self._arg(x, dot, scopes) if isinstance(x, tuple) else x
                res = v
                if name == "and" and not truthy(v):
                    return v
                if name == "or" and truthy(v):
                    return v
            return res
        fn = self.funcs.get(name)
        if fn is None:
            raise TemplateError(f"function {name!r} not defined")
        vals = [self._arg(x, dot, scopes) for x in args]
        if has_prev:
            vals.append(prev)
        return fn(*vals)

    def _pipe(self, p: Pipeline, dot, scopes):
        val = None
        has = False
        for cmd in p.cmds:
            if not cmd:
                raise TemplateError("empty command")
            head = cmd[0]
            if head[0] == "ident" and head[1] not in ("true", "false", "nil"):
                val = self._call(head[1], cmd[1:], dot, scopes, val, has)
            else:
                if len(cmd) > 1:
                    raise TemplateError(f"can't give arguments to non-function {head}")
                val = self._arg(head, dot, scopes)
                if has:
                    raise TemplateError("non-function in pipeline")
            has = True
        if p.decl:
            if len(p.decl) == 1:
                self._set_var(p.decl[0], val, scopes, not p.is_assign)
            return None if not p.is_assign else None
        return val

    def _exec(self, nodes, dot, scopes, out):
        for n in nodes:
            if isinstance(n, Text):
                out.append(n.text)
            elif isinstance(n, Action):
                v = self._pipe(n.pipe, dot, scopes)
                if not n.pipe.decl:
                    out.append(_go_str(v) if v is not None else "<no value>")
            elif isinstance(n, If):
                done = False
                for pipe, body in n.branches:
                    scopes.append({})
                    v = self._pipe(pipe, dot, scopes) if not pipe.decl else self._decl_val(pipe, dot, scopes)
                    if truthy(v):
                        self._exec(body, dot, scopes, out)
                        scopes.pop()
                        done = True
                        break
                    scopes.pop()
                if not done and n.else_ is not None:
                    self._exec(n.else_, dot, scopes, out)
            elif isinstance(n, With):
                done = False
                for pipe, body in n.branches:
                    scopes.append({})
                    v = self._pipe(pipe, dot, scopes) if not pipe.decl else self._decl_val(pipe, dot, scopes)
                    if truthy(v):
                        self._exec(body, v, scopes, out)
                        scopes.pop()
                        done = True
                        break
                    scopes.pop()
                if not done and n.else_ is not None:
                    self._exec(n.else_, dot, scopes, out)
            elif isinstance(n, Range):
                self._range(n, dot, scopes, out)
            elif isinstance(n, TemplateCall):
                body = self.defines.get(n.name)
                if body is None:
                    raise TemplateError(f"no such template {n.name!r}")
                d = self._pipe(n.pipe, dot, scopes) if n.pipe else None
                self._exec(body, d, [{"$": d}], out)
            elif isinstance(n, Break):
                raise _Brk()
            elif isinstance(n, Continue):
                raise _Cont()

    def _decl_val(self, pipe, dot, scopes):
        p2 = Pipeline([], False, pipe.cmds)
        v = self._pipe(p2, dot, scopes)
        self._set_var(pipe.decl[0], v, scopes, True)
        return v

    def _range(self, n: Range, dot, scopes, out):
        p2 = Pipeline([], False, n.pipe.cmds)
        coll = self._pipe(p2, dot, scopes)
        if isinstance(coll, dict):
            items = sorted(coll.items(), key=lambda kv: str(kv[0]))
        elif isinstance(coll, int) and not isinstance(coll, bool):
            items = list(enumerate(range(coll)))
        elif coll is None:
            items = []
        else:
            items = list(enumerate(coll))
        if not items:
            if n.else_ is not None:
                self._exec(n.else_, dot, scopes, out)
            return
        for k, v in items:
            scopes.append({})
            if n.pipe.decl:
                if len(n.pipe.decl) == 1:
                    scopes[-1][n.pipe.decl[0]] = v
                else:
                    scopes[-1][n.pipe.decl[0]] = k
                    scopes[-1][n.pipe.decl[1]] = v
            try:
                self._exec(n.body, v, scopes, out)
            except _Cont:
                pass
            except _Brk:
                scopes.pop()
                break
            scopes.pop()


_cache: dict[str, Template] = {}


def render(src: str, data) -> str:
    t = _cache.get(src)
    if t is None:
        t = Template(src)
        if len(_cache) > 512:
            _cache.clear()
        _cache[src] = t
    return t.render(data)
