// Minimal chat client for dllama-api. Non-streaming replies read `generated_text` (the reference
// web-ui contract, web-ui/app.js:40) with the OpenAI `choices[0].message.content` as fallback;
// streaming replies consume the server-sent chat.completion.chunk events.
const API = `${location.origin}/v1`;
const log = document.getElementById('log');
const input = document.getElementById('input');
const form = document.getElementById('form');
const history = [];

function add(role, text) {
  const div = document.createElement('div');
  div.className = `msg ${role}`;
  div.textContent = text;
  log.appendChild(div);
  log.scrollTop = log.scrollHeight;
  return div;
}

function meta(div, text) {
  const m = document.createElement('span');
  m.className = 'meta';
  m.textContent = text;
  div.appendChild(m);
}

async function health() {
  try {
    const h = await (await fetch(`${location.origin}/health`)).json();
    document.getElementById('status').textContent =
      `${h.model} · ${h.backend} · ${h.nodes} node(s) · ${h.slots} slots · ${h.active} active`;
  } catch (e) {
    document.getElementById('status').textContent = 'server unreachable';
  }
}

async function send(text) {
  history.push({ role: 'user', content: text });
  add('user', text);
  const body = {
    messages: history,
    max_tokens: Number(document.getElementById('maxTokens').value),
    temperature: Number(document.getElementById('temperature').value),
    stream: document.getElementById('stream').checked,
  };
  const out = add('assistant', '');
  const t0 = performance.now();
  const res = await fetch(`${API}/chat/completions`, {
    method: 'POST', headers: { 'Content-Type': 'application/json' }, body: JSON.stringify(body),
  });
  if (!res.ok) throw new Error(`HTTP ${res.status}: ${await res.text()}`);
  let reply = '';
  let n = 0;
  if (body.stream) {
    const reader = res.body.getReader();
    const dec = new TextDecoder();
    let buf = '';
    for (;;) {
      const { value, done } = await reader.read();
      if (done) break;
      buf += dec.decode(value, { stream: true });
      let i;
      while ((i = buf.indexOf('\n\n')) >= 0) {
        const ev = buf.slice(0, i).trim();
        buf = buf.slice(i + 2);
        if (!ev.startsWith('data:')) continue;
        const data = ev.slice(5).trim();
        if (data === '[DONE]') continue;
        const delta = JSON.parse(data).choices[0].delta.content;
        if (delta) { reply += delta; n++; out.textContent = reply; log.scrollTop = log.scrollHeight; }
      }
    }
  } else {
    const data = await res.json();
    reply = data.generated_text || (data.choices && data.choices[0].message.content) || '';
    n = data.usage ? data.usage.completion_tokens : 0;
    out.textContent = reply;
  }
  const s = (performance.now() - t0) / 1000;
  meta(out, `${n} tokens · ${s.toFixed(2)} s · ${(n / s).toFixed(1)} tok/s`);
  history.push({ role: 'assistant', content: reply });
}

form.addEventListener('submit', async (e) => {
  e.preventDefault();
  const text = input.value.trim();
  if (!text) return;
  input.value = '';
  const btn = form.querySelector('button[type=submit]');
  btn.disabled = true;
  try { await send(text); } catch (err) { add('error', String(err)); }
  btn.disabled = false;
  health();
});
input.addEventListener('keydown', (e) => {
  if (e.key === 'Enter' && !e.shiftKey) { e.preventDefault(); form.requestSubmit(); }
});
document.getElementById('reset').addEventListener('click', () => { history.length = 0; log.innerHTML = ''; });
health();
