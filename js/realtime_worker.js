"use strict";
/*
 * realtime_worker.js -- the worker-thread seam of the reference
 * (src/services/worker/RealtimeWorkerImpl.ts:29-84) on the MI355X engine.
 *
 * The reference's realtime step runs in a Node `worker_threads` Worker: it
 * builds `new Traces(traces)`, runs combineLogsToRealtimeData + 
 * toCombinedRealtimeData and toEndpointDependencies, merges the cached graph
 * (`new EndpointDependencies(existingDep).combineWith(newDep)`), and posts
 * plain JSON arrays back (postMessage, RealtimeWorkerImpl.ts:74-81).  This
 * script does the same with NativeTraces: each Worker loads kmz.node into its
 * own context (the addon is context-aware, NAPI_MODULE_INIT) and owns its
 * kmz_ctx.  Message in: { uniqueId, traces | json (Uint8Array of Trace[][]),
 * logs?, replicas?, existingDep? }; out: { uniqueId, rlDataList, dependencies, ms }
 * or { uniqueId, error }.  `dependencies` is existingDep.combineWith(newDep)
 * (merged on columns) when existingDep is given, else the per-row JSON of
 * toEndpointDependencies().
 */
const { parentPort, workerData } = require("worker_threads");
const path = require("path");
const { NativeTraces, cache } = require(path.join(__dirname, "kmamiz_native"));

function step(msg) {
  const t0 = process.hrtime.bigint();
  const traces = msg.json ? NativeTraces.fromJSON(Buffer.from(msg.json), msg.device || 0)
                          : new NativeTraces(msg.traces, msg.device || 0);
  const rlDataList = traces.combineLogsToRealtimeData(msg.logs || [], msg.replicas).toCombinedRealtimeData();
  // RealtimeWorkerImpl.ts:67-70: with a cached graph the merge runs on columns
  // (the window's reduced graph from the engine's entry order, kmz_cache.js),
  // and only the merged rows (<= one per endpoint) become objects; the first
  // tick returns newDep itself, one row per span id, as the reference does
  const dependencies = msg.existingDep
    ? cache.ReducedDependencies.fromJSON(msg.existingDep, false).combineWith(traces.toReducedDependencies()).toJSON()
    : traces.toEndpointDependencies();
  return { uniqueId: msg.uniqueId, rlDataList, dependencies, ms: Number(process.hrtime.bigint() - t0) / 1e6 };
}

if (parentPort) {
  parentPort.on("message", (msg) => {
    try {
      parentPort.postMessage(step(msg));
    } catch (e) {
      parentPort.postMessage({ uniqueId: msg.uniqueId, error: String(e && e.stack ? e.stack : e) });
    }
  });
  if (workerData && workerData.ready) parentPort.postMessage({ ready: true });
}

module.exports = { step };
