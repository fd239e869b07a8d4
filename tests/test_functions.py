"""Tool-calling: output parsing (cases mirror pkg/functions/parse_test.go) and JSON-schema grammars
checked end-to-end through the native GBNF matcher (csrc/runtime/grammar.cpp)."""
import json

import pytest

from localai_tfp_amd import functions as F
from localai_tfp_amd.config.model_config import FunctionsConfig
from localai_tfp_amd.functions.grammar import GrammarOptions, schema_to_grammar


def fc(**kw):
    c = FunctionsConfig()
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def names_args(res):
    return [(r.name, r.arguments) for r in res]


def test_parse_plain_object():
    assert names_args(F.parse_function_call('{"name": "add", "arguments": {"x": 5, "y": 3}}', fc())) == \
        [("add", '{"x":5,"y":3}')]


@pytest.mark.parametrize("key", ["name", "function"])
def test_parse_response_regex(key):
    c = fc(response_regex=[rf"(?P<{key}>\w+)\s*\((?P<arguments>.*)\)"], function_name_key=key)
    assert names_args(F.parse_function_call('add({"x":5,"y":3})', c)) == [("add", '{"x":5,"y":3}')]


def test_parse_empty_and_invalid():
    assert F.parse_function_call("", fc()) == []
    assert F.parse_function_call("invalid input", fc()) == []


def test_parse_array_and_garbage():
    s = '[{"name": "add", "arguments": {"x": 5, "y": 3}}, {"name": "subtract", "arguments": {"x": 10, "y": 7}}]'
    assert names_args(F.parse_function_call(s, fc())) == [("add", '{"x":5,"y":3}'), ("subtract", '{"x":10,"y":7}')]
    s = '{"name": "add", "arguments": {"x": 5, "y": 3}} invalid {"name": "add", "arguments": {"x": 5, "y": 3}}'
    assert len(F.parse_function_call(s, fc())) == 2


def test_parse_function_name_key():
    c = fc(function_name_key="function")
    assert names_args(F.parse_function_call('{"function": "add", "arguments": {"x": 5, "y": 3}}', c)) == \
        [("add", '{"x":5,"y":3}')]


def test_parse_json_regex_match_repeated():
    s = ('Some text\n<tool_call>{"name": "add", "arguments": {"x": 5, "y": 3}}</tool_call>\n'
         '<tool_call>{"name": "subtract", "arguments": {"x": 10, "y": 7}}</tool_call>\nafter')
    c = fc(json_regex_match=[r"(?s)<tool_call>(.*?)</tool_call>"])
    assert names_args(F.parse_function_call(s, c)) == [("add", '{"x":5,"y":3}'), ("subtract", '{"x":10,"y":7}')]
    c = fc(json_regex_match=[r"(?s)(.*?)</tool_call>"])
    assert F.parse_function_call('{"name": "add", "arguments": {"x": 5, "y": 3}}</tool_call>', c)[0].name == "add"


def test_parse_single_quote_rewrites():
    s = "\nSome text before the JSON\n{'name': '\"add\"', 'arguments': {'x': 5, 'z': '\"v\"', 'y': 'v\"value\"'}}\nafter\n"
    c = fc(json_regex_match=[r"(?s)<tool_call>(.*?)</tool_call>"], replace_function_results=[
        {"key": r"(?s)^[^{\[]*", "value": ""},
        {"key": r"(?s)[^}\]]*$", "value": ""},
        {"key": r"'([^']*?)'", "value": r"_DQUOTE_${1}_DQUOTE_"},
        {"key": r'\\"', "value": "__TEMP_QUOTE__"},
        {"key": r'"', "value": r'\"'},
        {"key": r"\'", "value": "'"},
        {"key": r"_DQUOTE_", "value": '"'},
        {"key": r"__TEMP_QUOTE__", "value": '"'},
    ])
    res = F.parse_function_call(s, c)
    assert names_args(res) == [('"add"', r'{"x":5,"y":"v\"value\"","z":"\"v\""}')]


def test_llama31_format_and_argument_regex():
    res = F.parse_function_call('<function=get_weather>{"city": "Paris"}</function>', fc())
    assert names_args(res) == [("get_weather", '{"city":"Paris"}')]
    c = fc(response_regex=[r"(?P<name>\w+)\((?P<arguments>[^)]*)\)"],
           argument_regex=[r"(?P<key>\w+)=(?P<value>\w+)"])
    assert names_args(F.parse_function_call("move(x=1, y=two)", c)) == [("move", '{"x":"1","y":"two"}')]


def test_text_content_and_cleanup():
    s = "before\n<sketchpad>\nroses are red\n</sketchpad>\n<tool_call>{}</tool_call>"
    assert F.parse_text_content(s, fc(capture_llm_results=[r"(?s)<sketchpad>(.*?)</sketchpad>"])) == "roses are red"
    assert F.parse_text_content("nothing", fc(capture_llm_results=[r"(?s)<sketchpad>(.*?)</sketchpad>"])) == ""
    c = fc(replace_llm_results=[{"key": r"(?s)<think>.*?</think>", "value": ""}])
    assert F.cleanup_llm_result("<think>hmm</think>answer", c) == "answer"


def test_parse_json_objects():
    assert F.parse_json_objects('{"key1": "value1"} {"key2": "value2"}') == [{"key1": "value1"}, {"key2": "value2"}]
    assert F.parse_json_objects('[{"key1": "value1"}]') == [{"key1": "value1"}]
    assert F.parse_json_objects("invalid json") == []
    assert F.parse_json_objects('{"key1": "value1"} invalid {"key2": 2}') == [{"key1": "value1"}, {"key2": 2}]


def test_go_sub_expansions():
    assert F.go_sub(r"(?P<w>\w+)@(\w+)", "${2}:$w $$", "a@b") == "b:a $"
    assert F.go_sub(r"x", r"\n", "x") == "\\n"


# ------------------------------------------------------------------------------------------------
# grammar generation, validated by actually matching strings with the native GBNF engine

TOOLS = [
    {"type": "function", "function": {"name": "create_event", "parameters": {"type": "object", "properties": {
        "title": {"type": "string"}, "date": {"type": "string"}, "time": {"type": "string"}}}}},
    {"type": "function", "function": {"name": "search", "parameters": {"type": "object", "properties": {
        "query": {"type": "string"}}}}},
]


def _native():
    rn = pytest.importorskip("localai_tfp_amd.runtime_native")
    try:
        rn._rt()
    except Exception as ex:  # pragma: no cover - build environment problem
        pytest.skip(f"libmxrt unavailable: {ex}")
    return rn


def _accepts(gbnf: str, text: str) -> bool:
    rn = _native()
    g = rn.NativeGrammar(gbnf)
    tb = [bytes([i]) for i in range(256)]
    m = rn.GrammarMatcher(g, rn.NativeVocab(tb), tb)
    return m.accept_bytes(text.encode()) and m.is_done()


def test_tool_grammar_accepts_valid_calls():
    funcs = F.functions_from_request(None, TOOLS)
    g = F.grammar_for(funcs, fc())
    assert "root ::=" in g
    ok = '{"arguments": {"date": "d", "time": "t", "title": "x"}, "name": "create_event"}'
    assert _accepts(g, ok)
    assert _accepts(g, '{"arguments": {"query": "weather"}, "name": "search"}')
    assert not _accepts(g, '{"arguments": {"query": "weather"}, "name": "delete_all"}')
    assert not _accepts(g, "hello")


def test_tool_grammar_options():
    funcs = F.functions_from_request(None, TOOLS)
    call = '{"arguments": {"query": "q"}, "name": "search"}'
    c = fc()
    c.grammar.parallel_calls = True
    g = F.grammar_for(funcs, c)
    assert _accepts(g, "[\n" + call + ",\n" + call + "]")
    assert _accepts(g, call)
    c.grammar.mixed_mode = True
    g = F.grammar_for(funcs, c)
    assert _accepts(g, "just some text ")
    c = fc()
    c.grammar.prefix = "<tool>"
    g = F.grammar_for(funcs, c)
    assert _accepts(g, "<tool>" + call) and not _accepts(g, call)


def test_schema_types_and_llama31():
    schema = {"type": "object", "properties": {
        "n": {"type": "integer"}, "f": {"type": "number"}, "b": {"type": "boolean"},
        "e": {"enum": ["red", "green"]}, "l": {"type": "array", "items": {"type": "string"}}}}
    g = schema_to_grammar(schema)
    assert _accepts(g, json.dumps({"b": True, "e": "red", "f": -1.5e3, "l": ["a", "b"], "n": 42}))
    assert not _accepts(g, json.dumps({"b": True, "e": "blue", "f": 1, "l": [], "n": 1}))
    funcs = F.functions_from_request(None, TOOLS)
    g = schema_to_grammar(F.to_json_structure(funcs), GrammarOptions(schema_type="llama3.1"))
    assert _accepts(g, '<function=search>{"query": "x"}</function>')
    assert not _accepts(g, '<function=nope>{"query": "x"}</function>')


def test_json_object_grammar():
    assert _accepts(F.JSON_BNF, '{"a": [1, 2, {"b": null}], "c": "d"}')
    assert not _accepts(F.JSON_BNF, "[1, 2]")
