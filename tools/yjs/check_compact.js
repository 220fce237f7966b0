// TEST TOOLING ONLY: Yjs reference for store-based compaction (see check_compact.py).
// Per case: a fresh Y.Doc applies the updates in order (one transaction each, GC on), then
// encodeStateAsUpdate; the oracle's compaction is compared byte for byte and re-applied.
const fs = require('fs');
const Y = require('./yjs_load.js');
const rows = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const hex = h => Uint8Array.from(Buffer.from(h, 'hex'));
// canonical content of a document: per root type (doc.share, filled by integration), the
// sequence of live units (client, clock, value) in list order and the live map entries,
// nested types recursively; unit-level, so struct boundaries (merging) do not matter
const units = n => {
  const c = n.content;
  if (c.type) return [dumpType(c.type)];
  const v = c.getContent();
  return n.length === v.length ? v : [JSON.stringify(v)];
};
const dumpType = t => {
  const seq = [];
  for (let n = t._start; n !== null; n = n.right) {
    if (n.deleted) continue;
    const u = units(n);
    for (let i = 0; i < u.length; i++) seq.push([n.id.client, n.id.clock + i, u[i]]);
  }
  const map = [];
  for (const [k, n] of t._map) if (!n.deleted) map.push([k, n.id.client, n.id.clock, units(n)]);
  map.sort((a, b) => (a[0] < b[0] ? -1 : a[0] > b[0] ? 1 : 0));
  return { seq, map };
};
const json = d => {
  const o = {};
  for (const k of Array.from(d.share.keys()).sort()) o[k] = dumpType(d.share.get(k));
  return JSON.stringify(o);
};
const out = rows.map(r => { try { return check(r); } catch (e) { return { yjs_hex: '', byte_equal: false, content_equal: false, error: String(e) }; } });
function check(r) {
  const a = new Y.Doc();
  for (const u of r.updates) Y.applyUpdate(a, hex(u));
  const ya = Buffer.from(Y.encodeStateAsUpdate(a)).toString('hex');
  const b = new Y.Doc();
  Y.applyUpdate(b, hex(r.compact));
  const res = { yjs_hex: ya, byte_equal: ya === r.compact, content_equal: json(a) === json(b) };
  if (r.end !== undefined) res.text_equal = b.getText(r.root || 'text').toString() === r.end;
  return res;
}
process.stdout.write(JSON.stringify(out));
