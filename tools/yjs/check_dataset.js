// TEST TOOLING ONLY: applies oracle merges with the offline Yjs bundle (see check_dataset.py).
const fs = require('fs');
const Y = require('./yjs_load.js');
function norm(v) { // canonical JSON text: sorted keys, typed arrays as arrays
  if (v instanceof Uint8Array) return JSON.stringify(Array.from(v));
  if (Array.isArray(v)) return '[' + v.map(norm).join(',') + ']';
  if (v && typeof v === 'object') {
    return '{' + Object.keys(v).sort().map(k => JSON.stringify(k) + ':' + norm(v[k])).join(',') + '}';
  }
  return JSON.stringify(v === undefined ? null : v);
}
const rows = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const res = { text: 0, map: 0, array: 0, failures: [] };
rows.forEach((r, k) => {
  const d = new Y.Doc();
  const t = d.getText('text'), m = d.getMap('map'), a = d.getArray('array');
  Y.applyUpdate(d, Uint8Array.from(Buffer.from(r.merged, 'hex')));
  const okT = t.toString() === r.text, okM = norm(m.toJSON()) === norm(r.map), okA = norm(a.toJSON()) === norm(r.array);
  res.text += okT; res.map += okM; res.array += okA;
  if (!(okT && okM && okA)) res.failures.push(k);
});
process.stdout.write(JSON.stringify(res));
