"use strict";
// node js/run_fixture.js <Trace[][] json> [json] -> prints {rl, crl_rt, crl_tag, deps} as JSON
// ("json": through NativeTraces.fromJSON on the raw bytes)
// (driven by tests/test_gpu_node.py; needs a GPU)
const fs = require("fs");
const { NativeTraces } = require("./kmamiz_native");

const raw = fs.readFileSync(process.argv[2]);
const traces = JSON.parse(raw.toString("utf8"));
const t = process.argv[3] === "json" ? NativeTraces.fromJSON(raw, 0) : new NativeTraces(traces, 0);
const reps = [{ uniqueServiceName: "details\tbook\tv1", replicas: 3 }];
const out = {
  rl: t.toRealTimeData().toJSON(),
  crl_rt: t.toRealTimeData(reps).toCombinedRealtimeData(),
  crl_tag: t.combineLogsToRealtimeData([], reps).toCombinedRealtimeData(),
  deps: t.toEndpointDependencies(),
  info: NativeTraces.ToEndpointInfo(traces[0][0] || { name: "a.b.svc.c", tags: { "http.url": "x" }, timestamp: 0 }),
};
process.stdout.write(JSON.stringify(out));
