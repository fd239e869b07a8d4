"""JSON schema -> GBNF grammar (the grammar language llama.cpp and our engine/grammar.py accept).

Behavioural parity target: pkg/functions/grammars/json_schema.go (a port of llama.cpp's
json-schema-to-grammar) and llama31_schema.go (`<function=name>{...}</function>`), plus the
root-rewriting options of rules.go used for tool calling:
  maybe_array   - the model may emit a list of calls ("parallel_calls")
  maybe_string  - free text OR calls ("mixed_mode")
  prefix        - calls must start with a literal prefix
  no_mixed_free_string / disable_parallel_new_lines / expect_strings_after_json
Rules are emitted sorted by name for stable output.
"""
from __future__ import annotations

import json
import re
from dataclasses import dataclass

SPACE = '" "?'
PRIMITIVES = {
    "boolean": '("true" | "false") space',
    "number": '("-"? ([0-9] | [1-9] [0-9]*)) ("." [0-9]+)? ([eE] [-+]? [0-9]+)? space',
    "integer": '("-"? ([0-9] | [1-9] [0-9]*)) space',
    "string": '"\\"" ( [^"\\\\] | "\\\\" (["\\\\/bfnrt] | "u" [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F]) )* "\\"" space',
    "freestring": '( [^\\x00] | "\\\\" (["\\\\/bfnrt] | "u" [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F] [0-9a-fA-F]) )* space',
    "null": '"null" space',
}
# arbitrary JSON value (used when a schema says nothing: {"type": "object"} without properties)
VALUE_RULES = {
    "value": "object | array | string | number | boolean | null",
    "object": '"{" space ( string ":" space value ("," space string ":" space value)* )? "}" space',
    "array": '"[" space ( value ("," space value)* )? "]" space',
}
JSON_OBJECT_GBNF = "\n".join([
    "root ::= object",
    *(f"{k} ::= {v}" for k, v in VALUE_RULES.items() if k != "value"),
    "value ::= object | array | string | number | (\"true\" | \"false\" | \"null\") space",
    f"string ::= {PRIMITIVES['string']}",
    f"number ::= {PRIMITIVES['number']}",
    f"space ::= {SPACE}",
])
_BAD = re.compile(r"[^a-zA-Z0-9-]+")


def _lit(v) -> str:
    s = json.dumps(v, ensure_ascii=False)
    s = s.replace("\\", "\\\\").replace('"', '\\"').replace("\r", "\\r").replace("\n", "\\n")
    return f'"{s}"'


@dataclass
class GrammarOptions:
    maybe_array: bool = False
    maybe_string: bool = False
    prefix: str = ""
    no_mixed_free_string: bool = False
    disable_parallel_new_lines: bool = False
    expect_strings_after_json: bool = False
    prop_order: str = ""
    schema_type: str = ""  # "" (json) | "llama3.1"
    function_name_key: str = "name"


class SchemaConverter:
    def __init__(self, prop_order: str = ""):
        self.order = {n: i for i, n in enumerate(p for p in prop_order.split(",") if p)}
        self.rules: dict[str, str] = {"space": SPACE}

    def add(self, name: str, rule: str) -> str:
        key = _BAD.sub("-", name)
        if key in self.rules and self.rules[key] != rule:
            i = 0
            while f"{key}{i}" in self.rules:
                i += 1
            key = f"{key}{i}"
        self.rules[key] = rule
        return key

    def _ref(self, ref: str, root: dict) -> dict:
        for prefix in ("#/$defs/", "#/definitions/"):
            if ref.startswith(prefix):
                defs = root.get(prefix[2:-1], {})
                key = ref[len(prefix):]
                if key in defs:
                    return defs[key]
        raise ValueError(f"unresolvable $ref {ref}")

    def visit(self, schema: dict, name: str, root: dict) -> str:
        rn = name or "root"
        t = schema.get("type")
        if "oneOf" in schema or "anyOf" in schema:
            alts = schema.get("oneOf") or schema.get("anyOf") or []
            return self.add(rn, " | ".join(self.visit(a, f"{rn}-{i}", root) for i, a in enumerate(alts)))
        if "$ref" in schema:
            return self.visit(self._ref(schema["$ref"], root), name, root)
        if "const" in schema:
            return self.add(rn, _lit(schema["const"]))
        if "enum" in schema:
            return self.add(rn, " | ".join(_lit(v) for v in schema["enum"]))
        if isinstance(t, list):
            return self.add(rn, " | ".join(self.visit({**schema, "type": tt}, f"{rn}-{tt}", root) for tt in t))
        if t == "object" and isinstance(schema.get("properties"), dict) and schema["properties"]:
            props = list(schema["properties"].items())

            def key(kv):
                o = self.order.get(kv[0], 0)
                return (0 if o else 1, o, kv[0])
            if self.order:
                props.sort(key=key)
            else:
                props.sort(key=lambda kv: kv[0])
            parts = ['"{" space']
            for i, (pn, ps) in enumerate(props):
                sub = self.visit(ps if isinstance(ps, dict) else {}, f"{rn}-{pn}", root)
                if i:
                    parts.append('"," space')
                parts.append(f"{_lit(pn)} space \":\" space {sub}")
            parts.append('"}" space')
            return self.add(rn, " ".join(parts))
        if t == "object":
            for k, v in VALUE_RULES.items():
                self.rules.setdefault(k, v)
            for k in ("string", "number", "boolean", "null"):
                self.rules.setdefault(k, PRIMITIVES[k])
            return "object"
        if t == "array":
            items = schema.get("items")
            if isinstance(items, dict):
                it = self.visit(items, f"{rn}-item", root)
            else:
                for k, v in VALUE_RULES.items():
                    self.rules.setdefault(k, v)
                for k in ("string", "number", "boolean", "null"):
                    self.rules.setdefault(k, PRIMITIVES[k])
                it = "value"
            return self.add(rn, f'"[" space ({it} ("," space {it})*)? "]" space')
        if t is None:
            # untyped schema: any JSON value
            for k, v in VALUE_RULES.items():
                self.rules.setdefault(k, v)
            for k in ("string", "number", "boolean", "null"):
                self.rules.setdefault(k, PRIMITIVES[k])
            return self.add(rn, "value") if rn == "root" else "value"
        if t not in PRIMITIVES:
            raise ValueError(f"unsupported schema type {t!r}")
        return self.add("root" if rn == "root" else t, PRIMITIVES[t])

    def grammar(self, schema: dict, opts: GrammarOptions | None = None) -> str:
        self.add("freestring", PRIMITIVES["freestring"])
        self.visit(schema, "", schema)
        return rules_to_grammar(self.rules, opts or GrammarOptions())


def rules_to_grammar(rules: dict, o: GrammarOptions) -> str:
    swap = o.maybe_array or o.maybe_string or bool(o.prefix)
    lines = []
    for name in sorted(rules):
        n = "realvalue" if swap and name == "root" else name
        lines.append(f"{n} ::= {rules[name]}")
    if not swap:
        return "\n".join(lines)
    new_root = "arr | realvalue" if o.maybe_array else "realvalue"
    free = "freestring" if o.no_mixed_free_string else "mixedstring"
    if o.prefix:
        pre = o.prefix.replace("\n", "\\n")
        if o.maybe_array and o.maybe_string:
            new_root = f"({new_root})"
        if o.maybe_string:
            new_root = f'( "{pre}" {new_root} | {free} ) '
        else:
            new_root = f'"{pre}" {new_root}'
    elif o.maybe_string:
        new_root = f"{free} | {new_root}"
    lines.append(f"root ::= {new_root}")
    if o.disable_parallel_new_lines:
        lines.append('arr ::= "[" ( realvalue ("," realvalue)* )? "]"')
    else:
        lines.append('arr ::= "[\\n" ( realvalue (",\\n" realvalue)* )? "]"')
    if o.maybe_array:
        if o.expect_strings_after_json:
            lines.append("mixedstring ::= freestring | freestring arr freestring | (freestring realvalue freestring)* | realvalue | arr")
        else:
            lines.append("mixedstring ::= freestring | freestring arr | freestring realvalue | realvalue | arr")
    else:
        if o.expect_strings_after_json:
            lines.append("mixedstring ::= freestring | (freestring realvalue freestring)* | realvalue")
        else:
            lines.append("mixedstring ::= freestring | freestring realvalue | realvalue")
    return "\n".join(lines)


class Llama31Converter:
    """`<function=NAME>{"arg": ...}</function>` tool-call format (Llama 3.1 style)."""

    def __init__(self, name_key: str = "name"):
        self.name_key = name_key or "name"

    def grammar(self, schema: dict, opts: GrammarOptions | None = None) -> str:
        o = opts or GrammarOptions()
        sc = SchemaConverter(o.prop_order)
        alts = schema.get("oneOf") or schema.get("anyOf") or [schema]
        calls = []
        for i, alt in enumerate(alts):
            props = alt.get("properties", {})
            fname = props.get(self.name_key, {}).get("const")
            args = props.get("arguments", {"type": "object"})
            arg_rule = sc.visit(args, f"fn{i}-args", schema)
            calls.append(f'"<function={_esc_plain(fname)}>" {arg_rule} "</function>"')
        sc.rules["root"] = " | ".join(calls)
        sc.rules.setdefault("freestring", PRIMITIVES["freestring"])
        return rules_to_grammar(sc.rules, o)


def _esc_plain(s) -> str:
    return str(s).replace("\\", "\\\\").replace('"', '\\"')


def schema_to_grammar(schema: dict, opts: GrammarOptions | None = None) -> str:
    o = opts or GrammarOptions()
    if o.schema_type in ("llama3.1", "llama31", "llama-3.1"):
        return Llama31Converter(o.function_name_key).grammar(schema, o)
    return SchemaConverter(o.prop_order).grammar(schema, o)
