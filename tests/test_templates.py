"""Go-template interpreter + message templating. Expected strings are the reference's own
fixtures (pkg/templates/evaluator_test.go) for the llama3 / chatml chat_message templates."""
import pytest

from localai_tfp_amd.config.model_config import ModelConfig
from localai_tfp_amd.templates import gotemplate as G
from localai_tfp_amd.templates.evaluator import Evaluator

LLAMA3 = '''<|start_header_id|>{{if eq .RoleName "assistant"}}assistant{{else if eq .RoleName "system"}}system{{else if eq .RoleName "tool"}}tool{{else if eq .RoleName "user"}}user{{end}}<|end_header_id|>

{{ if .FunctionCall -}}
Function call:
{{ else if eq .RoleName "tool" -}}
Function response:
{{ end -}}
{{ if .Content -}}
{{.Content -}}
{{ else if .FunctionCall -}}
{{ toJson .FunctionCall -}}
{{ end -}}
<|eot_id|>'''

CHATML = '''<|im_start|>{{if eq .RoleName "assistant"}}assistant{{else if eq .RoleName "system"}}system{{else if eq .RoleName "tool"}}tool{{else if eq .RoleName "user"}}user{{end}}
{{- if .FunctionCall }}
<tool_call>
{{- else if eq .RoleName "tool" }}
<tool_response>
{{- end }}
{{- if .Content}}
{{.Content }}
{{- end }}
{{- if .FunctionCall}}
{{toJson .FunctionCall}}
{{- end }}
{{- if .FunctionCall }}
</tool_call>
{{- else if eq .RoleName "tool" }}
</tool_response>
{{- end }}<|im_end|>'''

GALAXY = "A long time ago in a galaxy far, far away..."


def _cfg(chat_message):
    c = ModelConfig()
    c.template.chat_message = chat_message
    return c


@pytest.mark.parametrize("tpl,msg,expected", [
    (LLAMA3, {"role": "user", "content": GALAXY, "string_content": GALAXY},
     "<|start_header_id|>user<|end_header_id|>\n\nA long time ago in a galaxy far, far away...<|eot_id|>"),
    (LLAMA3, {"role": "assistant", "content": GALAXY, "string_content": GALAXY},
     "<|start_header_id|>assistant<|end_header_id|>\n\nA long time ago in a galaxy far, far away...<|eot_id|>"),
    (LLAMA3, {"role": "assistant", "function_call": {"function": "test"}},
     "<|start_header_id|>assistant<|end_header_id|>\n\nFunction call:\n{\"function\":\"test\"}<|eot_id|>"),
    (LLAMA3, {"role": "tool", "content": "Response from tool", "string_content": "Response from tool"},
     "<|start_header_id|>tool<|end_header_id|>\n\nFunction response:\nResponse from tool<|eot_id|>"),
    (CHATML, {"role": "user", "content": GALAXY, "string_content": GALAXY},
     "<|im_start|>user\nA long time ago in a galaxy far, far away...<|im_end|>"),
    (CHATML, {"role": "assistant", "function_call": {"function": "test"}},
     "<|im_start|>assistant\n<tool_call>\n{\"function\":\"test\"}\n</tool_call><|im_end|>"),
    (CHATML, {"role": "tool", "content": "Response from tool", "string_content": "Response from tool"},
     "<|im_start|>tool\n<tool_response>\nResponse from tool\n</tool_response><|im_end|>"),
])
def test_reference_fixtures(tpl, msg, expected):
    ev = Evaluator("")
    assert ev.template_messages([msg], _cfg(tpl), [], False) == expected


def test_gotemplate_core():
    r = G.render
    assert r("{{.Input}}!", {"Input": "hi"}) == "hi!"
    assert r("a {{- \" b \" -}} c", {}) == "a b c"
    assert r("{{range $i, $m := .L}}{{$i}}={{$m}};{{end}}", {"L": ["x", "y"]}) == "0=x;1=y;"
    assert r("{{range .L}}{{.}}{{else}}empty{{end}}", {"L": []}) == "empty"
    assert r("{{with .A}}{{.B}}{{end}}", {"A": {"B": 3}}) == "3"
    assert r("{{if and .A (not .B)}}yes{{else}}no{{end}}", {"A": 1, "B": 0}) == "yes"
    assert r("{{printf \"%s-%d\" .S .N}}", {"S": "a", "N": 7}) == "a-7"
    assert r("{{ .S | upper | trim }}", {"S": " abc "}) == "ABC"
    assert r("{{toJson .M}}", {"M": {"a": [1, 2]}}) == '{"a":[1,2]}'
    assert r("{{$x := 1}}{{if eq $x 1}}one{{end}}", {}) == "one"
    assert r('{{define "T"}}[{{.}}]{{end}}{{template "T" .V}}', {"V": 5}) == "[5]"
    assert r("{{/* comment */}}ok", {}) == "ok"
    assert r("{{len .L}}", {"L": [1, 2, 3]}) == "3"
    assert r("{{index .M \"k\"}}", {"M": {"k": "v"}}) == "v"
    assert r("{{ default \"d\" .X }}", {}) == "d"
    assert r('{{ if hasPrefix "ab" .S }}p{{ end }}', {"S": "abc"}) == "p"
    assert r("{{range .L}}{{if eq . 2}}{{break}}{{end}}{{.}}{{end}}", {"L": [1, 2, 3]}) == "1"


def test_chat_and_function_templates():
    c = ModelConfig()
    c.template.chat_message = "<{{.RoleName}}>{{.Content}}"
    c.template.chat = "{{.Input}}\nASSISTANT:"
    c.template.function = "TOOLS:{{range .Functions}}{{.name}} {{end}}\n{{.Input}}"
    ev = Evaluator("")
    msgs = [{"role": "system", "content": "s", "string_content": "s"}, {"role": "user", "content": "u", "string_content": "u"}]
    assert ev.template_messages(msgs, c, [], False) == "<system>s\n<user>u\nASSISTANT:"
    out = ev.template_messages(msgs, c, [{"name": "f1"}, {"name": "f2"}], True)
    assert out.startswith("TOOLS:f1 f2 \n<system>s")


def test_roles_fallback_without_templates():
    c = ModelConfig()
    c.roles = {"user": "USER: ", "assistant": "ASSISTANT: "}
    msgs = [{"role": "user", "content": "hi", "string_content": "hi"}]
    assert Evaluator("").template_messages(msgs, c, [], False) == "USER: hi"


def test_tmpl_file_in_model_path(tmp_path):
    (tmp_path / "mytpl.tmpl").write_text("Q: {{.Input}}\nA:")
    c = ModelConfig()
    c.template.completion = "mytpl"
    ev = Evaluator(str(tmp_path))
    from localai_tfp_amd.templates.evaluator import COMPLETION
    assert ev.evaluate_for_prompt(COMPLETION, c, {"Input": "2+2"}) == "Q: 2+2\nA:"
