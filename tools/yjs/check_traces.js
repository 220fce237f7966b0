// TEST TOOLING ONLY: applies oracle trace merges with the offline Yjs bundle (see check_traces.py).
const fs = require('fs');
const Y = require('./yjs_load.js');
const rows = JSON.parse(fs.readFileSync(process.argv[2], 'utf8'));
const hex = h => Uint8Array.from(Buffer.from(h, 'hex'));
const out = rows.map(r => {
  const a = new Y.Doc();
  Y.applyUpdate(a, hex(r.merged));
  const b = new Y.Doc();
  Y.applyUpdate(b, hex(r.half));
  Y.applyUpdate(b, hex(r.diff));
  return { text_equal: a.getText('text').toString() === r.end,
           diff_text_equal: b.getText('text').toString() === r.end };
});
process.stdout.write(JSON.stringify(out));
