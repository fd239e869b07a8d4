"""Minimal web UI (parity target: core/http/routes/ui.go:62-572 — index, chat, text2image, tts,
talk, model browser, p2p pages). Self-contained HTML + vanilla JS over the public API."""
from __future__ import annotations

import html

from fastapi import APIRouter, Request
from fastapi.responses import HTMLResponse

from .openai import app_of

router = APIRouter()

_CSS = ("body{font-family:system-ui,sans-serif;margin:0;background:#111;color:#eee}"
        "nav{background:#222;padding:10px}nav a{color:#8cf;margin-right:14px;text-decoration:none}"
        "main{padding:16px;max-width:960px;margin:auto}textarea,input,select{width:100%;background:#1b1b1b;"
        "color:#eee;border:1px solid #333;padding:6px}button{background:#246;color:#fff;border:0;padding:8px 14px;"
        "margin-top:6px;cursor:pointer}.msg{white-space:pre-wrap;border-bottom:1px solid #222;padding:6px}"
        "table{border-collapse:collapse;width:100%}td,th{border-bottom:1px solid #333;padding:4px;text-align:left}")
_NAV = ('<nav><a href="/">Home</a><a href="/chat">Chat</a><a href="/text2image">Images</a><a href="/tts">TTS</a>'
        '<a href="/talk">Talk</a><a href="/browse">Models</a><a href="/p2p">P2P</a></nav>')


def _page(title: str, body: str) -> HTMLResponse:
    return HTMLResponse(f"<!doctype html><html><head><meta charset=utf-8><title>{html.escape(title)}</title>"
                        f"<style>{_CSS}</style></head><body>{_NAV}<main>{body}</main></body></html>")


def _model_select(a, sel: str = "") -> str:
    opts = "".join(f'<option {"selected" if n == sel else ""}>{html.escape(n)}</option>' for n in a.list_models())
    return f'<select id="model">{opts}</select>'


@router.get("/")
async def index(request: Request):
    a = app_of(request)
    rows = "".join(f"<tr><td>{html.escape(c.name)}</td><td>{html.escape(c.backend or 'auto')}</td>"
                   f"<td>{'loaded' if a.loader.get(c.name) else ''}</td></tr>" for c in a.configs.all())
    loose = "".join(f"<li>{html.escape(f)}</li>" for f in a.configs.loose_model_files())
    return _page("LocalAI", f"<h2>Installed models</h2><table><tr><th>name</th><th>backend</th><th>state</th></tr>"
                             f"{rows}</table><h3>Model files without config</h3><ul>{loose}</ul>")


# All page scripts build DOM nodes with createElement/textContent: model output, user input and gallery
# metadata (remote, untrusted) are never parsed as HTML (the reference renders through Go's
# auto-escaping html/template).
_JS_UTIL = """
function el(tag,text,cls){const e=document.createElement(tag);if(text!==undefined)e.textContent=text;if(cls)e.className=cls;return e;}
function msgDiv(who,text){const d=el('div',undefined,'msg');const b=el('b',who+': ');const s=el('span',text);d.appendChild(b);d.appendChild(s);return [d,s];}
async function streamChat(model,msgs,onText){const r=await fetch('/v1/chat/completions',{method:'POST',
headers:{'Content-Type':'application/json'},body:JSON.stringify({model:model,messages:msgs,stream:true})});
const rd=r.body.getReader();const dec=new TextDecoder();let acc='',buf='';
for(;;){const {done,value}=await rd.read();if(done)break;buf+=dec.decode(value,{stream:true});let i;
while((i=buf.indexOf('\\n\\n'))>=0){const line=buf.slice(0,i);buf=buf.slice(i+2);if(!line.startsWith('data: '))continue;
const p=line.slice(6);if(p==='[DONE]')continue;const j=JSON.parse(p);
const c=j.choices&&j.choices[0]&&j.choices[0].delta&&j.choices[0].delta.content;if(c){acc+=c;onText(acc);}}}return acc;}
"""


@router.get("/chat")
@router.get("/chat/{model}")
async def chat_page(request: Request, model: str = ""):
    a = app_of(request)
    js = _JS_UTIL + """
const log=document.getElementById('log');let msgs=[];
async function send(){const t=document.getElementById('in');const m=document.getElementById('model').value;
msgs.push({role:'user',content:t.value});log.appendChild(msgDiv('you',t.value)[0]);t.value='';
const [d,span]=msgDiv('ai','');log.appendChild(d);
const acc=await streamChat(m,msgs,x=>{span.textContent=x;});msgs.push({role:'assistant',content:acc});}
document.getElementById('send').addEventListener('click',send);
"""
    return _page("Chat", f"<h2>Chat</h2>{_model_select(a, model)}<div id=log></div>"
                         f"<textarea id=in rows=3></textarea><button id=send>Send</button><script>{js}</script>")


@router.get("/text2image")
@router.get("/text2image/{model}")
async def t2i_page(request: Request, model: str = ""):
    a = app_of(request)
    js = _JS_UTIL + """async function gen(){const r=await fetch('/v1/images/generations',{method:'POST',
headers:{'Content-Type':'application/json'},body:JSON.stringify({model:document.getElementById('model').value,
prompt:document.getElementById('p').value,size:'512x512'})});const j=await r.json();
const out=document.getElementById('out');out.replaceChildren();
for(const d of (j.data||[])){const im=el('img');im.width=512;im.src=d.url||('data:image/png;base64,'+d.b64_json);out.appendChild(im);}}
document.getElementById('go').addEventListener('click',gen);"""
    return _page("Images", f"<h2>Text to image</h2>{_model_select(a, model)}<input id=p placeholder=prompt>"
                           f"<button id=go>Generate</button><div id=out></div><script>{js}</script>")


@router.get("/tts")
@router.get("/tts/{model}")
async def tts_page(request: Request, model: str = ""):
    a = app_of(request)
    js = """async function say(){const r=await fetch('/tts',{method:'POST',headers:{'Content-Type':'application/json'},
body:JSON.stringify({model:document.getElementById('model').value,input:document.getElementById('t').value})});
const b=await r.blob();const au=document.getElementById('au');au.src=URL.createObjectURL(b);au.play();}
document.getElementById('go').addEventListener('click',say);"""
    return _page("TTS", f"<h2>Text to speech</h2>{_model_select(a, model)}<input id=t>"
                        f"<button id=go>Speak</button><audio id=au controls></audio><script>{js}</script>")


@router.get("/talk")
async def talk_page(request: Request):
    """Record -> /v1/audio/transcriptions -> /v1/chat/completions -> /tts (core/http/views/talk.html)."""
    a = app_of(request)
    names = a.list_models()

    def sel(i):
        return f'<select id="{i}">' + "".join(f"<option>{html.escape(n)}</option>" for n in names) + "</select>"
    js = _JS_UTIL + """
let rec=null,chunks=[];const log=document.getElementById('log');const msgs=[];
async function start(){const st=await navigator.mediaDevices.getUserMedia({audio:true});rec=new MediaRecorder(st);
chunks=[];rec.ondataavailable=e=>chunks.push(e.data);rec.onstop=turn;rec.start();}
function stop(){if(rec)rec.stop();}
async function turn(){const fd=new FormData();fd.append('file',new Blob(chunks),'talk.webm');
fd.append('model',document.getElementById('stt').value);
const tr=await (await fetch('/v1/audio/transcriptions',{method:'POST',body:fd})).json();const text=tr.text||'';
log.appendChild(msgDiv('you',text)[0]);msgs.push({role:'user',content:text});
const [d,span]=msgDiv('ai','');log.appendChild(d);
const ans=await streamChat(document.getElementById('llm').value,msgs,x=>{span.textContent=x;});
msgs.push({role:'assistant',content:ans});
const r=await fetch('/tts',{method:'POST',headers:{'Content-Type':'application/json'},
body:JSON.stringify({model:document.getElementById('voice').value,input:ans})});
const au=document.getElementById('au');au.src=URL.createObjectURL(await r.blob());au.play();}
document.getElementById('rec').addEventListener('click',start);document.getElementById('stop').addEventListener('click',stop);
"""
    return _page("Talk", f"<h2>Talk</h2><p>Transcription {sel('stt')} LLM {sel('llm')} Voice {sel('voice')}</p>"
                         f"<button id=rec>Record</button><button id=stop>Stop &amp; send</button>"
                         f"<div id=log></div><audio id=au controls></audio><script>{js}</script>")


@router.get("/browse")
async def browse_page(request: Request):
    """Gallery browser with install progress (core/http/routes/ui.go /browse + elements/gallery.go):
    install posts /models/apply and polls /models/jobs/<uuid> until processed."""
    js = _JS_UTIL + """
async function load(){const r=await fetch('/models/available');const ms=await r.json();const tb=document.getElementById('g');
tb.replaceChildren();for(const m of ms){const tr=el('tr');tr.appendChild(el('td',m.name));
tr.appendChild(el('td',m.description||''));const td=el('td');const b=el('button','install');
b.dataset.id=(m.gallery&&m.gallery.name?m.gallery.name+'@':'')+m.name;const st=el('span','');
b.addEventListener('click',()=>inst(b.dataset.id,st,b));td.appendChild(b);td.appendChild(st);tr.appendChild(td);tb.appendChild(tr);}}
async function inst(id,st,b){b.disabled=true;const r=await fetch('/models/apply',{method:'POST',
headers:{'Content-Type':'application/json'},body:JSON.stringify({id:id})});const j=await r.json();
for(;;){await new Promise(res=>setTimeout(res,1000));const s=await (await fetch('/models/jobs/'+encodeURIComponent(j.uuid))).json();
const pct=s.progress!==undefined?Math.round(s.progress)+'%':'';st.textContent=' '+(s.message||'')+' '+pct;
if(s.processed||s.error){st.textContent=s.error?' error: '+s.error:' installed';b.disabled=false;break;}}}
load();"""
    return _page("Models", f"<h2>Model gallery</h2><table id=g></table><script>{js}</script>")


@router.get("/p2p")
async def p2p_page(request: Request):
    a = app_of(request)
    return _page("P2P", f"<h2>Distributed inference</h2><p>Token: <code>{html.escape(a.cfg.p2p_token or '-')}"
                        "</code></p><p>Nodes: see <a href='/api/p2p'>/api/p2p</a></p>")
