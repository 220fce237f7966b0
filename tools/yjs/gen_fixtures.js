// TEST TOOLING ONLY: generates tests/golden/yjs_fixtures.json with the offline
// Yjs bundle (see yjs_load.js).  Each case holds input v1 updates plus Yjs's own
// mergeUpdates / diffUpdate / encodeStateVectorFromUpdate outputs.  Yjs is a
// semantic cross-check, not a bit-exact yrs oracle (SURVEY.md Appendix E): the
// tests compare against it only for cases flagged `agree`.
//   node tools/yjs/gen_fixtures.js > tests/golden/yjs_fixtures.json
const Y = require('./yjs_load.js');

let seed = 0x9E3779B9;
function rnd() { // xorshift32, deterministic
  seed ^= seed << 13; seed >>>= 0; seed ^= seed >>> 17; seed ^= seed << 5; seed >>>= 0;
  return seed / 4294967296;
}
function ri(n) { return Math.floor(rnd() * n); }
const hex = u => Buffer.from(u).toString('hex');
const cases = [];

function newDoc(client, gc = true) {
  const d = new Y.Doc({ gc });
  d.clientID = client;
  return d;
}
function record(name, updates, agree, extraSvs = []) {
  const merged = Y.mergeUpdates(updates);
  const svs = [new Uint8Array([0]), Y.encodeStateVectorFromUpdate(merged), ...extraSvs];
  const c = {
    name, agree,
    updates: updates.map(hex),
    yjs_merge: hex(merged),
    yjs_sv: hex(Y.encodeStateVectorFromUpdate(merged)),
    diffs: svs.map(sv => ({ sv: hex(sv), yjs: hex(Y.diffUpdate(merged, sv)) })),
  };
  cases.push(c);
}
function typing(doc, text, nOps, delFrac, chars = 'abcdefgh') {
  for (let i = 0; i < nOps; i++) {
    const len = text.length;
    if (len > 0 && rnd() < delFrac) {
      const p = ri(len), k = 1 + ri(Math.min(5, len - p));
      text.delete(p, k);
    } else {
      let s = '';
      const k = 1 + ri(8);
      for (let j = 0; j < k; j++) s += chars[ri(chars.length)];
      text.insert(ri(len + 1), s);
    }
  }
}

// 1) single client per-op typing, merged in order / reversed / shuffled / with duplicates
for (const [nOps, del] of [[20, 0], [60, 0.2], [150, 0.35]]) {
  const d = newDoc(100 + nOps);
  const ups = [];
  d.on('update', u => ups.push(u));
  typing(d, d.getText('text'), nOps, del);
  record(`single_typing_${nOps}`, ups, true);
  record(`single_typing_${nOps}_rev`, ups.slice().reverse(), true);
  const sh = ups.slice();
  for (let i = sh.length - 1; i > 0; i--) { const j = ri(i + 1); [sh[i], sh[j]] = [sh[j], sh[i]]; }
  record(`single_typing_${nOps}_shuf`, sh, true);
  record(`single_typing_${nOps}_dup`, ups.concat(ups.slice(0, ups.length >> 1)), true);
}

// 2) 2-4 synced replicas, each op one update (config-2 style)
for (const nc of [2, 3, 4]) {
  const docs = [], ups = [];
  for (let c = 0; c < nc; c++) docs.push(newDoc(1000 * (c + 1) + nc));
  docs.forEach((d, i) => d.on('update', (u, origin) => { if (origin !== 'sync') ups.push(u); }));
  for (let i = 0; i < 80; i++) {
    const d = docs[ri(nc)];
    typing(d, d.getText('text'), 1, 0.2);
    const u = ups[ups.length - 1];
    docs.forEach(o => { if (o !== d) Y.applyUpdate(o, u, 'sync'); });
  }
  record(`synced_${nc}clients`, ups, false); // DS with several clients: hash order differs
  record(`synced_${nc}clients_inserts_only_head`, ups.slice(0, 10), nc === 1);
}

// 3) concurrent (unsynced) clients then merge
{
  const a = newDoc(7), b = newDoc(9), ups = [];
  a.on('update', u => ups.push(u)); b.on('update', u => ups.push(u));
  typing(a, a.getText('text'), 30, 0.1); typing(b, b.getText('text'), 30, 0.1);
  record('concurrent_2', ups, false);
}

// 4) snapshot + overlapping per-op log (partial overlaps -> exact path)
for (const gc of [true, false]) {
  const d = newDoc(4242 + (gc ? 1 : 0), gc), ups = [];
  d.on('update', u => ups.push(u));
  const t = d.getText('text');
  typing(d, t, 40, 0.3);
  const snap1 = Y.encodeStateAsUpdate(d);
  typing(d, t, 40, 0.3);
  const snap2 = Y.encodeStateAsUpdate(d);
  record(`snapshot_plus_log_gc${gc}`, [snap1].concat(ups), true);
  record(`log_plus_snapshot_gc${gc}`, ups.concat([snap2]), true);
  record(`two_snapshots_gc${gc}`, [snap1, snap2], true);
  record(`snapshot_mid_log_gc${gc}`, ups.slice(0, 20).concat([snap1], ups.slice(20)), true);
  const sv1 = Y.encodeStateVectorFromUpdate(snap1);
  record(`snap_diff_gc${gc}`, [snap1, Y.diffUpdate(snap2, sv1)], true, [sv1]);
}

// 5) maps, arrays with Any values, xml, nested types
{
  const d = newDoc(555), ups = [];
  d.on('update', u => ups.push(u));
  const m = d.getMap('map');
  m.set('a', 1); m.set('b', 'str'); m.set('a', 2); m.set('c', true); m.set('d', null);
  m.set('e', [1, 2, 'x']); m.set('f', -7); m.set('g', 1.5); m.set('h', 2147483647); m.set('i', -2147483648);
  m.set('j', new Uint8Array([1, 2, 3]));
  const arr = d.getArray('array');
  arr.insert(0, [1, 'two', false, null, [3, [4]], -1, 123456]);
  arr.delete(1, 2);
  arr.insert(2, ['z']);
  record('map_array_any', ups, false);
  const x = d.getXmlFragment('xml');
  const el = new Y.XmlElement('p');
  x.insert(0, [el]);
  el.insert(0, [new Y.XmlText('hello')]);
  el.setAttribute('class', 'c1');
  const nested = new Y.Map();
  m.set('nested', nested);
  nested.set('k', 'v');
  record('map_array_xml_nested', ups, false);
}

// 6) numbers outside int31 / floats (yrs canonicalises differently from Yjs)
{
  const d = newDoc(777), ups = [];
  d.on('update', u => ups.push(u));
  const arr = d.getArray('array');
  arr.insert(0, [3e9, 0.1, 1e300, -0.0, 2 ** 53, 2 ** 53 + 2, 1e-7, 255.5, Number.MAX_SAFE_INTEGER]);
  record('numbers', ups, false);
}

// 7) rich text with formatting / embeds (Format items -> unsupported in round 1)
{
  const d = newDoc(888), ups = [];
  d.on('update', u => ups.push(u));
  const t = d.getText('text');
  t.insert(0, 'hello world');
  t.format(0, 5, { bold: true });
  t.insertEmbed(3, { image: 'x.png' });
  record('rich_text', ups, false);
}

// 8) utf-16 surrogates and multi-byte text, snapshot overlap forces splits inside strings
{
  const d = newDoc(999, false), ups = [];
  d.on('update', u => ups.push(u));
  const t = d.getText('text');
  t.insert(0, 'a😀bé€c');
  t.insert(2, 'XY');
  t.insert(5, '😀😀');
  const snap = Y.encodeStateAsUpdate(d);
  t.insert(1, 'Q');
  record('utf16_text', ups, true);
  record('utf16_snapshot_overlap', [snap].concat(ups), true);
  record('utf16_log_then_snapshot', ups.concat([snap]), true);
}

// 9) subdocument and move-less large deletes
{
  const d = newDoc(31337, true), ups = [];
  d.on('update', u => ups.push(u));
  const t = d.getText('text');
  t.insert(0, 'x'.repeat(300));
  t.delete(10, 250);
  t.insert(5, 'yy');
  const snap = Y.encodeStateAsUpdate(d);
  record('big_delete_gc', ups, true);
  record('big_delete_gc_snapshot_first', [snap].concat(ups), true);
  const sub = d.getMap('subdocs');
  sub.set('child', new Y.Doc({ guid: 'child-guid-1' }));
  record('subdoc', ups, false);
}

process.stdout.write(JSON.stringify({ generator: 'Yjs ^13.5 (JupyterLab offline bundle) via tools/yjs/gen_fixtures.js', cases }, null, 0));
