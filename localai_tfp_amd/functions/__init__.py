"""OpenAI functions/tools support (reference: pkg/functions/functions.go:14-98,
function_structure.go:9-43, parse.go:16-373, json_mode.go).

* `Function` / `Tool` request types, `to_json_structure` (tools -> a oneOf JSON schema whose
  members are {"name": const, "arguments": {...}}), `select`;
* `grammar_for(...)` builds the GBNF constraining the model to emit such calls (functions/grammar.py);
* `parse_function_call` / `parse_text_content` / `cleanup_llm_result` recover the calls from
  model output: regex extraction, then lenient multi-object JSON scanning.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass, field

from .grammar import JSON_OBJECT_GBNF, GrammarOptions, schema_to_grammar  # noqa: F401

JSON_BNF = JSON_OBJECT_GBNF


@dataclass
class Function:
    name: str = ""
    description: str = ""
    strict: bool = False
    parameters: dict = field(default_factory=dict)

    @classmethod
    def from_dict(cls, d: dict) -> "Function":
        return cls(d.get("name", ""), d.get("description", ""), bool(d.get("strict", False)),
                   d.get("parameters") or {})

    def to_dict(self) -> dict:
        return {"name": self.name, "description": self.description, "strict": self.strict,
                "parameters": self.parameters}


@dataclass
class FuncCallResult:
    name: str
    arguments: str


def functions_from_request(functions: list | None, tools: list | None) -> list[Function]:
    out = [Function.from_dict(f) for f in (functions or [])]
    for t in tools or []:
        if t.get("type", "function") == "function" and t.get("function"):
            out.append(Function.from_dict(t["function"]))
    return out


def to_json_structure(funcs: list[Function], name_key: str = "", args_key: str = "") -> dict:
    nk = name_key or "name"
    ak = args_key or "arguments"
    one_of = []
    defs = None
    for f in funcs:
        props = (f.parameters or {}).get("properties") or {}
        if defs is None and (f.parameters or {}).get("$defs"):
            defs = f.parameters["$defs"]
        one_of.append({"type": "object", "properties": {
            nk: {"const": f.name},
            ak: {"type": "object", "properties": props},
        }})
    js = {"oneOf": one_of}
    if defs:
        js["$defs"] = defs
    return js


def select(funcs: list[Function], name: str) -> list[Function]:
    for f in funcs:
        if f.name == name:
            return [f]
    return []


def grammar_options(fc) -> GrammarOptions:
    """FunctionsConfig -> GrammarOptions (parse.go GrammarOptions)."""
    g = fc.grammar
    return GrammarOptions(
        maybe_array=g.parallel_calls, maybe_string=g.mixed_mode, prefix=g.prefix,
        no_mixed_free_string=g.no_mixed_free_string, disable_parallel_new_lines=g.disable_parallel_new_lines,
        expect_strings_after_json=g.expect_strings_after_json, prop_order=g.properties_order,
        schema_type=g.schema_type, function_name_key=fc.function_name_key or "name")


def grammar_for(funcs: list[Function], fc) -> str:
    js = to_json_structure(funcs, fc.function_name_key, fc.function_arguments_key)
    return schema_to_grammar(js, grammar_options(fc))


# ------------------------------------------------------------------------------------------------
# parsing model output


def _pairs(items):
    """replace_* config entries: list of {key: ..., value: ...} (or [k, v])."""
    for it in items or []:
        if isinstance(it, dict):
            yield it.get("key", ""), it.get("value", "")
        elif isinstance(it, (list, tuple)) and len(it) == 2:
            yield it[0], it[1]


_GO_REPL = re.compile(r"\$(?:\{(\w+)\}|(\w+)|\$)")


def go_sub(pattern: str, repl: str, s: str) -> str:
    """regexp.ReplaceAllString semantics: `$1`, `${1}`, `${name}` expand, `$$` is a literal `$`,
    backslashes in the replacement are literal."""
    def expand(m):
        def sub(g):
            if g.group(0) == "$$":
                return "$"
            key = g.group(1) or g.group(2)
            try:
                v = m.group(int(key)) if key.isdigit() else m.group(key)
            except IndexError:
                v = ""
            return v or ""
        return _GO_REPL.sub(sub, repl)
    return re.sub(pattern, expand, s)



def _marshal(v) -> str:
    # encoding/json.Marshal: map keys sorted, compact, non-ASCII kept
    return json.dumps(v, ensure_ascii=False, separators=(",", ":"), sort_keys=True)


def cleanup_llm_result(s: str, fc) -> str:
    for k, v in _pairs(fc.replace_llm_results):
        s = go_sub(k, v, s)
    return s


def parse_text_content(s: str, fc) -> str:
    for r in fc.capture_llm_results or []:
        m = re.search(r, s, re.S)
        if m and m.groups():
            return m.group(1).strip()
    return ""


def parse_json_objects(s: str) -> list[dict]:
    """All JSON objects in `s`, skipping garbage between them ({..} junk {..} -> two objects);
    a top-level array contributes its object members."""
    dec = json.JSONDecoder()
    out = []
    i = 0
    n = len(s)
    while i < n:
        j = min((p for p in (s.find("{", i), s.find("[", i)) if p >= 0), default=-1)
        if j < 0:
            break
        try:
            obj, end = dec.raw_decode(s, j)
        except json.JSONDecodeError:
            i = j + 1
            continue
        if isinstance(obj, dict):
            out.append(obj)
        elif isinstance(obj, list):
            out.extend(o for o in obj if isinstance(o, dict))
        i = end
    return out


def _escape_newlines_in_strings(s: str) -> str:
    # the reference escapes raw newlines before JSON decoding (utils.EscapeNewLines)
    out = []
    in_str = False
    esc = False
    for ch in s:
        if in_str:
            if esc:
                esc = False
            elif ch == "\\":
                esc = True
            elif ch == '"':
                in_str = False
            elif ch == "\n":
                out.append("\\n")
                continue
        elif ch == '"':
            in_str = True
        out.append(ch)
    return "".join(out)


def parse_function_call_args(args: str, fc) -> str:
    if not fc.argument_regex:
        return args
    kn = fc.argument_regex_key_name or "key"
    vn = fc.argument_regex_value_name or "value"
    res = {}
    for r in fc.argument_regex:
        for m in re.finditer(r, args):
            gd = m.groupdict()
            if kn in gd and vn in gd:
                res[gd[kn]] = gd[vn]
    return _marshal(res)


def parse_function_call(s: str, fc) -> list[FuncCallResult]:
    for k, v in _pairs(fc.replace_function_results):
        s = go_sub(k, v, s)
    nk = fc.function_name_key or "name"
    ak = fc.function_arguments_key or "arguments"
    results: list[FuncCallResult] = []
    if fc.response_regex:
        for r in fc.response_regex:
            for m in re.finditer(r, s, re.S):
                gd = m.groupdict()
                name = gd.get(nk, "")
                if not name:
                    return results
                results.append(FuncCallResult(name, parse_function_call_args(gd.get(ak, ""), fc)))
        return results
    candidates = []
    for r in fc.json_regex_match or []:
        ms = [m.group(1) for m in re.finditer(r, s, re.S) if m.groups()]
        if ms:
            candidates.extend(ms)
            break
    if not candidates:
        candidates = [s]
    # llama3.1 format: <function=name>{json}</function>
    for c in list(candidates):
        for m in re.finditer(r"<function=([^>]+)>(.*?)</function>", c, re.S):
            try:
                args = json.loads(m.group(2))
            except json.JSONDecodeError:
                args = m.group(2)
            results.append(FuncCallResult(m.group(1), _marshal(args) if not isinstance(args, str) else args))
    if results:
        return results
    for c in candidates:
        for obj in parse_json_objects(_escape_newlines_in_strings(c)):
            name = obj.get(nk)
            if not isinstance(name, str) or ak not in obj:
                continue
            args = obj[ak]
            results.append(FuncCallResult(name, _marshal(args)))
    return results
