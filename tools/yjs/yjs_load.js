// TEST TOOLING ONLY (this container): loads the Yjs ^13.5 bundle that ships
// inside JupyterLab's static assets so it can generate realistic v1 updates and
// cross-check merge semantics.  Never shipped, never run on the GPU box.
const fs = require('fs');
const path = require('path');
const STATIC = '/opt/conda/share/jupyter/lab/static';
const WANT = ['73502', '14247', '15966', '20817', '29194', '48307', '58290', '59735',
  '64485', '65679', '7049', '72382', '90421', '97027'];
global.self = global;
const mods = {};
self.webpackChunk_jupyterlab_application_top = {
  push: ([ids, m]) => Object.assign(mods, m)
};
for (const f of fs.readdirSync(STATIC)) {
  if (!f.endsWith('.js')) continue;
  const src = fs.readFileSync(path.join(STATIC, f), 'utf8');
  if (!WANT.some(id => src.includes(id + ':') || src.includes('"' + id + '"'))) continue;
  try { new Function('self', src)(self); } catch (e) { /* not a chunk */ }
}
const cache = {};
function n(id) {
  id = String(id);
  if (cache[id]) return cache[id].exports;
  const m = cache[id] = { exports: {} };
  if (!mods[id]) throw new Error('missing module ' + id);
  mods[id](m, m.exports, n);
  return m.exports;
}
n.r = e => { Object.defineProperty(e, '__esModule', { value: true }); };
n.d = (e, d) => { for (const k in d) if (!Object.prototype.hasOwnProperty.call(e, k)) Object.defineProperty(e, k, { enumerable: true, get: d[k] }); };
n.o = (o, p) => Object.prototype.hasOwnProperty.call(o, p);
n.n = m => { const g = m && m.__esModule ? () => m.default : () => m; n.d(g, { a: g }); return g; };
n.g = global;
global.crypto = { getRandomValues: a => (require('crypto').randomFillSync(a), a) };
module.exports = n('73502');
