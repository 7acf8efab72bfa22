"use strict";
// node tools/bench_ingest_node.js <Trace[][] json file> -> one JSON line:
// the reference's own ingest cost in Node (JSON.parse + the object ingest of
// js/kmamiz_native.js) vs NativeTraces.fromJSON's (kmz_parse_zipkin) on the bytes.
const fs = require("fs");
const path = require("path");
const { ingest, ingestJSON } = require(path.join(__dirname, "..", "js", "kmamiz_native"));

const raw = fs.readFileSync(process.argv[2]);
const sec = (f) => {
  let best = 1e9;
  for (let r = 0; r < 3; r++) {
    const t = process.hrtime.bigint();
    f();
    best = Math.min(best, Number(process.hrtime.bigint() - t) / 1e9);
  }
  return best;
};
let n = 0;
const tObj = sec(() => {
  n = ingest(JSON.parse(raw.toString("utf8"))).spans.span_id.length;
});
const tNat = sec(() => ingestJSON(raw, 0));
process.stdout.write(
  JSON.stringify({
    node_json_parse_plus_ingest_spans_per_s: Math.round(n / tObj),
    node_native_json_spans_per_s: Math.round(n / tNat),
    node_speedup: Math.round((tObj / tNat) * 10) / 10,
  }) + "\n"
);
