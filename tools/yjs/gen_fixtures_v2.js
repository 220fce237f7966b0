// TEST TOOLING ONLY: lib0 v2 fixtures from the offline Yjs bundle (see yjs_load.js).
// Every scenario records the same edits twice — v1 updates (doc.on('update')) and v2
// updates (doc.on('updateV2')) — plus Yjs's mergeUpdatesV2 / encodeStateVectorFromUpdateV2
// / diffUpdateV2 outputs.  Yjs is a semantic cross-check, not a bit-exact yrs oracle
// (SURVEY.md App. E): tests compare bytes with it only where the case says `agree`.
//   node tools/yjs/gen_fixtures_v2.js > tests/golden/yjs_fixtures_v2.json
const Y = require('./yjs_load.js');

let seed = 0x2545F491;
function rnd() {
  seed ^= seed << 13; seed >>>= 0; seed ^= seed >>> 17; seed ^= seed << 5; seed >>>= 0;
  return seed / 4294967296;
}
function ri(n) { return Math.floor(rnd() * n); }
const hex = u => Buffer.from(u).toString('hex');
const cases = [];

function newDoc(client) {
  const d = new Y.Doc();
  d.clientID = client;
  return d;
}
function watch(d) {
  const v1 = [], v2 = [];
  d.on('update', u => v1.push(u));
  d.on('updateV2', u => v2.push(u));
  return { v1, v2 };
}
function record(name, rec, agree) {
  const merged = Y.mergeUpdatesV2(rec.v2);
  const svs = [Y.encodeStateVectorFromUpdateV2(Y.mergeUpdatesV2(rec.v2.slice(0, rec.v2.length >> 1))),
               Y.encodeStateVectorFromUpdateV2(merged)];
  cases.push({
    name, agree,
    v1: rec.v1.map(hex), v2: rec.v2.map(hex),
    yjs_merge: hex(merged),
    yjs_sv: hex(Y.encodeStateVectorFromUpdateV2(merged)),
    diffs: svs.map(sv => ({ sv: hex(sv), yjs: hex(Y.diffUpdateV2(merged, sv)) })),
  });
}
function typing(text, nOps, delFrac, chars = 'abcdefgh') {
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
function shuffled(a) {
  const s = a.slice();
  for (let i = s.length - 1; i > 0; i--) { const j = ri(i + 1); [s[i], s[j]] = [s[j], s[i]]; }
  return s;
}

// 1) single-client typing (strings, deletes): in order, reversed, shuffled
for (const [nOps, del] of [[20, 0], [80, 0.25], [200, 0.35]]) {
  const d = newDoc(700 + nOps);
  const rec = watch(d);
  typing(d.getText('text'), nOps, del);
  record(`v2_typing_${nOps}`, rec, true);
  record(`v2_typing_${nOps}_rev`, { v1: rec.v1.slice().reverse(), v2: rec.v2.slice().reverse() }, true);
  const idx = shuffled([...rec.v1.keys()]);
  record(`v2_typing_${nOps}_shuf`, { v1: idx.map(i => rec.v1[i]), v2: idx.map(i => rec.v2[i]) }, true);
}
// 2) UTF-16: astral characters and accents (string column UTF-16 lengths)
{
  const d = newDoc(991);
  const rec = watch(d);
  typing(d.getText('text'), 60, 0.2, ['a', 'é', '€', '😀', '𝄞', 'b']);
  record('v2_utf16', rec, true);
}
// 3) map sets with repeated keys (parent_sub strings), nested types, Any values
{
  const d = newDoc(4242);
  const rec = watch(d);
  const m = d.getMap('map');
  for (let i = 0; i < 40; i++) {
    const k = 'k' + ri(6);
    const r = ri(4);
    if (r === 0) m.set(k, ri(1000));
    else if (r === 1) m.set(k, 'v' + ri(100));
    else if (r === 2) m.set(k, [true, null, ri(50)]);
    else m.set(k, new Y.Map());
  }
  record('v2_map', rec, false);
}
// 4) arrays of Any, deletes
{
  const d = newDoc(5151);
  const rec = watch(d);
  const a = d.getArray('arr');
  for (let i = 0; i < 50; i++) {
    if (a.length > 2 && rnd() < 0.3) a.delete(ri(a.length - 1), 1);
    else a.insert(ri(a.length + 1), [ri(100), 'x' + ri(9)]);
  }
  record('v2_array', rec, true);
}
// 5) rich text: formats and embeds (Format keys through the key table, JSON values as Any)
{
  const d = newDoc(6262);
  const rec = watch(d);
  const t = d.getText('text');
  typing(t, 30, 0.1);
  for (let i = 0; i < 12; i++) {
    const len = t.length;
    if (len < 2) break;
    const p = ri(len - 1);
    t.format(p, 1 + ri(Math.min(4, len - p - 1)), [{ bold: true }, { italic: true }, { color: '#' + ri(999) }][ri(3)]);
    if (rnd() < 0.3) t.insertEmbed(ri(t.length + 1), { image: 'img' + ri(9) + '.png' });
  }
  record('v2_rich_text', rec, false);
}
// 6) xml elements with attributes (TypeRef key table)
{
  const d = newDoc(7373);
  const rec = watch(d);
  const f = d.getXmlFragment('xml');
  for (let i = 0; i < 10; i++) {
    const e = new Y.XmlElement(['p', 'div', 'span'][ri(3)]);
    f.insert(f.length, [e]);
    e.setAttribute('id', 'e' + i);
    if (rnd() < 0.5) e.setAttribute('class', 'c' + ri(3));
    const tx = new Y.XmlText();
    e.insert(0, [tx]);
    tx.insert(0, 'hello ' + i);
  }
  record('v2_xml', rec, false);
}
// 7) two clients editing concurrently, synced by updates (multi-client sections)
{
  const a = newDoc(11), b = newDoc(22);
  const ra = watch(a), rb = watch(b);
  for (let r = 0; r < 6; r++) {
    typing(a.getText('text'), 10, 0.2);
    typing(b.getText('text'), 10, 0.2);
    Y.applyUpdateV2(b, Y.encodeStateAsUpdateV2(a, Y.encodeStateVector(b)));
    Y.applyUpdateV2(a, Y.encodeStateAsUpdateV2(b, Y.encodeStateVector(a)));
  }
  record('v2_two_clients', { v1: ra.v1.concat(rb.v1), v2: ra.v2.concat(rb.v2) }, false);
}
process.stdout.write(JSON.stringify({ generator: 'tools/yjs/gen_fixtures_v2.js', cases }));
