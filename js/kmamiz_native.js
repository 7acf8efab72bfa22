"use strict";
/*
 * kmamiz_native.js -- Node side of the drop-in boundary (SURVEY.md 8b seam 1).
 *
 * Turns KMamiz's `Trace[][]` into the columnar batch of include/kmz.h,
 * calls the MI355X engine through the N-API addon (kmz.node), and returns
 * the exact objects the reference's methods return:
 *
 *   NativeTraces#toRealTimeData(replicas)            Traces.ts:27-53
 *   NativeTraces#combineLogsToRealtimeData([], reps) Traces.ts:55-106 (no-log case)
 *   NativeRealtimeDataList#toCombinedRealtimeData()  RealtimeDataList.ts:22-97
 *   NativeTraces#toEndpointDependencies()            Traces.ts:112-211
 *   NativeTraces.ToEndpointInfo(trace)               Traces.ts:213-241
 *
 * The results are plain TRealtimeData / TCombinedRealtimeData /
 * TEndpointDependency arrays.  Integration (INTEGRATION.md) wraps them in the
 * reference's own RealtimeDataList / CombinedRealtimeDataList /
 * EndpointDependencies classes, whose merge and service-level methods run
 * unchanged.
 *
 * Node 12 compatible (no ?. / ??).
 */
const path = require("path");
const addon = require(path.join(__dirname, "kmz.node"));
const cache = require(path.join(__dirname, "kmz_cache"));

const KIND_SERVER = 1;
const KIND_CLIENT = 2;
const NONE32 = 0xffffffff;
const NONE64 = BigInt("0xffffffffffffffff");
const SHAPE_TAGS = [
  "http.method",
  "http.url",
  "istio.canonical_revision",
  "istio.canonical_service",
  "istio.namespace",
  "istio.mesh_id",
];

// Utils.ExplodeUrl (Utils.ts:83-106): [host, port, path(, service, namespace, clusterName)]
function explodeUrl(url, isServiceUrl) {
  if (url.search(/[a-z]+:\/\//) === -1) url = "://" + url;
  const m = url.match(/:\/\/([^:/]*)([:0-9]*)(.*)/) || [];
  const out = [m[1], m[2], m[3]];
  if (isServiceUrl) {
    const s = m[1].match(/(.*).svc[.]*(.*)/) || [];
    if (s[1]) {
      const cut = s[1].lastIndexOf(".");
      out.push(s[1].slice(0, cut), s[1].slice(cut + 1), s[2] || "cluster.local");
    }
  }
  return out;
}

function tagsOf(key) {
  const t = {};
  for (let i = 0; i < SHAPE_TAGS.length; i++) t[SHAPE_TAGS[i]] = key[i + 1];
  return t;
}

// identity rules, evaluated once per distinct shape
const RULES = {
  rt(key) {
    const ex = explodeUrl(key[0], true);
    const t = tagsOf(key);
    const usn = `${ex[3]}\t${ex[4]}\t${t["istio.canonical_revision"]}`;
    return {
      service: ex[3],
      namespace: ex[4],
      version: t["istio.canonical_revision"],
      method: t["http.method"],
      uniqueServiceName: usn,
      uniqueEndpointName: `${usn}\t${t["http.method"]}\t${t["http.url"]}`,
    };
  },
  tag(key) {
    const t = tagsOf(key);
    const usn = `${t["istio.canonical_service"]}\t${t["istio.namespace"]}\t${t["istio.canonical_revision"]}`;
    return {
      service: t["istio.canonical_service"],
      namespace: t["istio.namespace"],
      version: t["istio.canonical_revision"],
      method: t["http.method"],
      uniqueServiceName: usn,
      uniqueEndpointName: `${usn}\t${t["http.method"]}\t${t["http.url"]}`,
    };
  },
  dep(key) {
    const t = tagsOf(key);
    const u = explodeUrl(t["http.url"]);
    const ex = explodeUrl(key[0], true);
    let service = ex[3], namespace = ex[4], clusterName = ex[5];
    if (!key[0].includes(".svc.")) {
      service = t["istio.canonical_service"];
      namespace = t["istio.namespace"];
      clusterName = t["istio.mesh_id"];
    }
    const version = t["istio.canonical_revision"] || "NONE";
    const usn = `${service}\t${namespace}\t${version}`;
    return {
      version,
      service,
      namespace,
      url: t["http.url"],
      host: u[0],
      path: u[2],
      port: u[1] || "80",
      clusterName,
      method: t["http.method"],
      uniqueServiceName: usn,
      uniqueEndpointName: `${usn}\t${t["http.method"]}\t${t["http.url"]}`,
    };
  },
};

const HEX16 = /^[0-9a-f]{16}$/;

// Trace[][] -> columnar batch + dictionaries
function ingest(traces) {
  const flat = [];
  for (const t of traces) for (const s of t) flat.push(s);
  const n = flat.length;
  const sid = new BigUint64Array(n), pid = new BigUint64Array(n);
  const kind = new Uint8Array(n), shape = new Uint32Array(n), status = new Uint16Array(n);
  const duration = new Uint32Array(n), timestamp = new BigInt64Array(n);
  const shapeIndex = new Map(), shapes = [];
  const statusIndex = new Map(), statuses = [];
  const canonical = new Set(), other = new Map();
  const pendSid = [], pendPid = [];
  const idOf = (v, i, pend) => {
    if (typeof v === "string" && HEX16.test(v) && v !== "0000000000000000") {
      const x = BigInt("0x" + v);
      canonical.add(x);
      return x;
    }
    if (!other.has(v)) other.set(v, 0n);
    pend.push([i, v]);
    return 0n;
  };
  for (let i = 0; i < n; i++) {
    const s = flat[i];
    const tags = s.tags || {};
    sid[i] = idOf(s.id, i, pendSid);
    if (s.parentId) pid[i] = idOf(s.parentId, i, pendPid);
    kind[i] = s.kind === "SERVER" ? KIND_SERVER : s.kind === "CLIENT" ? KIND_CLIENT : 0;
    const key = [s.name].concat(SHAPE_TAGS.map((k) => tags[k]));
    const hk = JSON.stringify(key.map((v) => (v === undefined ? { u: 1 } : v)));
    let si = shapeIndex.get(hk);
    if (si === undefined) {
      si = shapes.length;
      shapeIndex.set(hk, si);
      shapes.push(key);
    }
    shape[i] = si;
    const st = tags["http.status_code"];
    let k = statusIndex.get(st);
    if (k === undefined) {
      k = statuses.length;
      statusIndex.set(st, k);
      statuses.push(st);
    }
    status[i] = k;
    if (!Number.isInteger(s.duration) || s.duration < 0 || s.duration >= 2 ** 32)
      throw new RangeError(`span ${i}: duration ${s.duration} is not an integer number of microseconds`);
    if (!Number.isInteger(s.timestamp)) throw new RangeError(`span ${i}: timestamp is not an integer`);
    duration[i] = s.duration;
    timestamp[i] = BigInt(s.timestamp);
  }
  // non-canonical ids: values no canonical id of the batch uses
  let next = 1n;
  for (const key of other.keys()) {
    while (canonical.has(next)) next++;
    other.set(key, next++);
  }
  for (const [i, v] of pendSid) sid[i] = other.get(v);
  for (const [i, v] of pendPid) pid[i] = other.get(v);
  return Object.assign(
    { flat, spans: { span_id: sid, parent_id: pid, kind, shape, status, duration, timestamp, index_base: 0 } },
    identities(shapes, statuses)
  );
}

// identities per shape and rule (errors kept, raised only when used)
function identities(shapes, statuses) {
  const ident = {}, epOf = {}, epNames = {}, poison = {};
  for (const rule of ["rt", "tag", "dep"]) {
    const names = new Map();
    ident[rule] = [];
    epOf[rule] = new Uint32Array(shapes.length);
    epNames[rule] = [];
    poison[rule] = new Map();
    shapes.forEach((key, i) => {
      let f, err;
      try {
        f = RULES[rule](key);
      } catch (e) {
        err = e;
      }
      ident[rule].push(f);
      let e;
      if (err) {
        e = epNames[rule].length;
        epNames[rule].push(null);
        poison[rule].set(e, err);
      } else {
        e = names.get(f.uniqueEndpointName);
        if (e === undefined) {
          e = epNames[rule].length;
          names.set(f.uniqueEndpointName, e);
          epNames[rule].push(f.uniqueEndpointName);
        }
      }
      epOf[rule][i] = e;
    });
  }
  return {
    shapesTable: {
      rt_ep: epOf.rt,
      tag_ep: epOf.tag,
      dep_ep: epOf.dep,
      n_rt_ep: epNames.rt.length,
      n_tag_ep: epNames.tag.length,
      n_dep_ep: epNames.dep.length,
      n_status: Math.max(1, statuses.length),
    },
    statuses,
    ident,
    poison,
    epNames,
  };
}

// Raw Zipkin response bytes (a Buffer of Trace[][] JSON) -> the same batch as
// ingest(JSON.parse(buf)), through the native parser (kmz_parse_zipkin,
// SURVEY.md 8f row 1); null when the batch is outside its fast path.  Span
// objects are parsed only if a per-span result needs them (`flat`).
function ingestJSON(buf, threads) {
  const r = addon.parseZipkin(buf, threads || 0);
  if (r === null) return null;
  const n = r.n;
  // every raw field slice decoded by one JSON.parse
  const sf = r.shapeFields, tf = r.statusFields;
  const parts = [];
  const collect = (f) => {
    for (let i = 0; i < f.length; i += 2) if (f[i + 1] >= 0) parts.push(buf.toString("utf8", f[i], f[i] + f[i + 1]));
  };
  collect(sf);
  collect(tf);
  const dec = JSON.parse("[" + parts.join(",") + "]");
  let k = 0;
  const next = (f, i) => (f[2 * i + 1] >= 0 ? dec[k++] : undefined);
  // raw shapes -> shapes by content, in first-occurrence order (as ingest numbers them)
  const nRaw = sf.length / 14, smap = new Uint32Array(nRaw);
  const shapeIndex = new Map(), shapes = [];
  for (let i = 0; i < nRaw; i++) {
    const key = [];
    for (let j = 0; j < 7; j++) key.push(next(sf, 7 * i + j));
    const hk = JSON.stringify(key.map((v) => (v === undefined ? { u: 1 } : v)));
    let si = shapeIndex.get(hk);
    if (si === undefined) {
      si = shapes.length;
      shapeIndex.set(hk, si);
      shapes.push(key);
    }
    smap[i] = si;
  }
  const nRawSt = tf.length / 2, tmap = new Uint32Array(nRawSt);
  const statusIndex = new Map(), statuses = [];
  for (let i = 0; i < nRawSt; i++) {
    const st = next(tf, i);
    let si = statusIndex.get(st);
    if (si === undefined) {
      si = statuses.length;
      statusIndex.set(st, si);
      statuses.push(st);
    }
    tmap[i] = si;
  }
  if (statuses.length > 65535) throw new RangeError("more than 65535 distinct status strings");
  const shape = new Uint32Array(n), status = new Uint16Array(n);
  for (let i = 0; i < n; i++) {
    shape[i] = smap[r.shape[i]];
    status[i] = tmap[r.status[i]];
  }
  const out = Object.assign(
    {
      spans: {
        span_id: r.span_id,
        parent_id: r.parent_id,
        kind: r.kind,
        shape,
        status,
        duration: r.duration,
        timestamp: r.timestamp,
        index_base: 0,
      },
    },
    identities(shapes, statuses)
  );
  let flat = null;
  Object.defineProperty(out, "flat", {
    get() {
      if (!flat) {
        flat = [];
        for (const t of JSON.parse(buf.toString("utf8"))) for (const s of t) flat.push(s);
      }
      return flat;
    },
  });
  return out;
}

function strip(o) {
  const r = {};
  for (const k of Object.keys(o)) if (o[k] !== undefined) r[k] = o[k];
  return r;
}

function replicaOf(replicas, usn) {
  if (!replicas) return undefined;
  const r = replicas.find((x) => x.uniqueServiceName === usn);
  return r ? r.replicas : undefined;
}

class NativeTraces {
  constructor(traces, device) {
    this._tv = traces;
    this._device = device || 0;
    this._b = null;
    this._ctx = null;
    this._raw = null;
  }
  // Traces of a raw Zipkin response (Buffer of Trace[][] JSON, as
  // ZipkinService.ts:44-57 receives it when asked for the bytes): the columns
  // come from the native parser; objects are built only when needed.
  static fromJSON(buf, device, threads) {
    const t = new NativeTraces(null, device);
    t._raw = buf;
    t._threads = threads || 0;
    return t;
  }
  get _traces() {
    if (this._tv === null && this._raw) this._tv = JSON.parse(this._raw.toString("utf8"));
    return this._tv;
  }
  toJSON() {
    return this._traces;
  }
  _batch() {
    if (!this._b) this._b = (this._raw && ingestJSON(this._raw, this._threads)) || ingest(this._traces);
    return this._b;
  }
  _engine() {
    if (!this._ctx) {
      const b = this._batch();
      this._ctx = addon.create(this._device);
      addon.load(this._ctx, b.spans, b.shapesTable);
    }
    return this._ctx;
  }
  toRealTimeData(replicas) {
    return new NativeRealtimeDataList(this, "rt", replicas);
  }
  // Traces.ts:55-106: stats from the engine; the Envoy-log join (59-84) adds
  // bodies and content types on the host (SURVEY.md 8f row 3)
  combineLogsToRealtimeData(structuredLogs, replicas) {
    return new NativeRealtimeDataList(this, "tag", replicas, logMap(structuredLogs));
  }
  toEndpointDependencies() {
    const b = this._batch();
    const ctx = this._engine();
    addon.run(ctx, addon.RUN_DEPS | addon.RUN_SPAN_LINKS);
    const n = b.spans.span_id.length;
    const links = addon.spanLinks(ctx, n);
    const E = b.shapesTable.n_dep_ep;
    const ep = new DataView(addon.endpoints(ctx, E));
    const dep = b.shapesTable.dep_ep;
    const info = (i) => {
      const f = b.ident.dep[b.spans.shape[i]];
      if (!f) throw b.poison.dep.get(dep[b.spans.shape[i]]);
      return strip(Object.assign({}, f, { timestamp: Number(b.spans.timestamp[i]) / 1000 }));
    };
    const rows = [];
    for (let i = 0; i < n; i++) if (links.rowpos[i] !== NONE64) rows.push(i);
    rows.sort((a, c) => (links.rowpos[a] < links.rowpos[c] ? -1 : 1));
    const lower = new Map();
    const uppers = rows.map((s) => {
      const chain = [];
      for (let q = links.cparent[s], d = 1; q !== NONE32; q = links.cparent[q], d++) {
        chain.push([q, d]);
        if (!lower.has(q)) lower.set(q, []);
        lower.get(q).push([s, d]);
      }
      return chain;
    });
    // new EndpointDependencies(dependencies) (Traces.ts:210): the constructor's
    // deprecation filter (EndpointDependencies.ts:44-74)
    return cache.filterOutDeprecatedRows(rows.map((s, r) => {
      const by = uppers[r].map(([q, d]) => ({ endpoint: info(q), distance: d, type: "CLIENT" }));
      const seen = new Map();
      for (const [t, d] of lower.get(s) || []) seen.set(`${dep[b.spans.shape[t]]}\t${d}`, [t, d]);
      const on = [...seen.values()].map(([t, d]) => ({ endpoint: info(t), distance: d, type: "SERVER" }));
      const e = dep[b.spans.shape[s]];
      const last = ep.getBigInt64(e * 24, true);
      const lastMs = Number(last) / 1000;
      return {
        endpoint: info(s),
        lastUsageTimestamp: lastMs > 0 ? lastMs : 0,
        isDependedByExternal: by.length === 0,
        dependingBy: by,
        dependingOn: on,
      };
    }));
  }
  // Service-level tail of the reduced graph (EndpointDependencies([]).combineWith(deps).trim()),
  // from the GPU's per-service counters (kmz_tail_run): toServiceInstability
  // (EndpointDependencies.ts:614-641), toServiceCoupling (643-657, RiskAnalyzer.ts:145-169),
  // the relying factor (RiskAnalyzer.ts:124-137) and cohesion's numbers (565-612), services
  // in first-row order.  labelMap: uniqueEndpointName -> labelName (EndpointDependencies.label()).
  serviceTail(labelMap) {
    const b = this._batch();
    const ctx = this._engine();
    addon.run(ctx, addon.RUN_DEPS);
    const E = b.shapesTable.n_dep_ep;
    const fields = new Array(E).fill(null);
    b.shapesTable.dep_ep.forEach((e, sh) => {
      if (b.ident.dep[sh]) fields[e] = b.ident.dep[sh];
    });
    const svcIdx = new Map(), clsIdx = new Map(), lsvcIdx = new Map(), lsvcOfCls = [];
    const svc = new Uint32Array(E), cls = new Uint32Array(E);
    const str = (x) => (x === undefined ? "undefined" : `${x}`);
    fields.forEach((f, e) => {
      const usn = f ? f.uniqueServiceName : "";
      const label = labelMap && f ? labelMap[f.uniqueEndpointName] : undefined;
      if (!svcIdx.has(usn)) svcIdx.set(usn, svcIdx.size);
      svc[e] = svcIdx.get(usn);
      const ck = `${usn}\t${str(f ? f.method : undefined)}\t${str(label)}`;
      if (!clsIdx.has(ck)) {
        clsIdx.set(ck, clsIdx.size);
        const l3 = usn.split("\t").slice(0, 3).join("\t");
        if (!lsvcIdx.has(l3)) lsvcIdx.set(l3, lsvcIdx.size);
        lsvcOfCls.push(lsvcIdx.get(l3));
      }
      cls[e] = clsIdx.get(ck);
    });
    const r = addon.serviceTail(ctx, { svc, cls, lsvc: Uint32Array.from(lsvcOfCls), n_svc: svcIdx.size,
                                       n_lsvc: lsvcIdx.size });
    const names = [...svcIdx.keys()];
    const ep = new DataView(addon.endpoints(ctx, E));
    const first = new Map(), total = new Array(names.length).fill(0), gateway = new Array(names.length).fill(false);
    for (let e = 0; e < E; e++) {
      if (!ep.getUint32(e * 24 + 20, true)) continue;  // has_row
      const v = svc[e], fr = ep.getBigUint64(e * 24 + 8, true);
      if (!first.has(v) || fr < first.get(v)) first.set(v, fr);
      total[v]++;
      if (!r.hasIn[e]) gateway[v] = true;
    }
    const order = [...first.keys()].sort((a, c) => (first.get(a) < first.get(c) ? -1 : 1));
    const st = (v, k) => r.stats[v * 8 + k];
    return order.map((v) => {
      const usn = names[v];
      const [s, n, ver] = usn.split("\t");
      const by = st(v, 0), on = st(v, 1), ais = st(v, 2) + (gateway[v] ? 1 : 0), ads = st(v, 3);
      let relying = gateway[v] ? 1 : 0;
      for (let d = 1; d < r.nDist; d++) relying += r.byDist[v * r.nDist + d] / d;
      const ncons = st(v, 4);
      return {
        uniqueServiceName: usn,
        name: `${s}.${n} (${ver})`,
        dependingBy: by,
        dependingOn: on,
        instability: on + by === 0 ? 0 : on / (on + by),
        ais,
        ads,
        acs: ais * ads,
        relyingFactor: relying,
        totalEndpoints: total[v],
        consumers: ncons,
        endpointUsageCohesion: ncons && total[v] ? st(v, 5) / total[v] / ncons : 0,
      };
    });
  }
  // EndpointDependencies([]).combineWith(this.toEndpointDependencies()).trim()
  // as cache columns (kmz_cache.ReducedDependencies), from the engine's entry
  // order (kmz_get_dep_entries): no object per row or entry.  `reg`: the
  // registry of the cache it will merge into (RealtimeWorkerImpl.ts:67-70).
  toReducedDependencies(reg) {
    const b = this._batch();
    const ctx = this._engine();
    addon.run(ctx, addon.RUN_DEPS | addon.RUN_DEP_ORDER);
    const E = b.shapesTable.n_dep_ep;
    const dep = addon.depEntries(ctx, E);
    const ep = addon.endpoints(ctx, E);
    const shapeFields = (sh) => {
      const f = b.ident.dep[sh];
      if (!f) throw b.poison.dep.get(b.shapesTable.dep_ep[sh]);
      return f;
    };
    return cache.ReducedDependencies.fromWindow(dep, ep, b.epNames.dep, shapeFields, reg);
  }
  static ToEndpointInfo(trace) {
    const tags = trace.tags || {};
    const key = [trace.name].concat(SHAPE_TAGS.map((k) => tags[k]));
    return strip(Object.assign(RULES.dep(key), { timestamp: trace.timestamp / 1000 }));
  }
}

// traceId -> spanId -> structured log trace (Traces.ts:59-67)
function logMap(structuredLogs) {
  const m = new Map();
  (structuredLogs || []).forEach((l) => {
    if (l.traces.length === 0) return;
    const { traceId } = l.traces[0];
    if (!m.has(traceId)) m.set(traceId, new Map());
    l.traces.forEach((t) => m.get(traceId).set(t.spanId, t));
  });
  return m.size ? m : null;
}

const JSON_CT = "application/json";

// Utils.Merge / MergeStringBody (Utils.ts:279-309), restated in the same language
function mergeValues(a, b) {
  if (Array.isArray(a) && Array.isArray(b)) return [...a.slice(0, 10), ...b.slice(0, 10)];
  if (!Array.isArray(a) && !Array.isArray(b)) return { ...a, ...b };
  return a || b;
}
function mergeStringBody(a, b) {
  if (a && b) {
    let pa, pb;
    try { pa = JSON.parse(a); } catch (e) {}
    try { pb = JSON.parse(b); } catch (e) {}
    if (pa && pb) return JSON.stringify(mergeValues(pa, pb));
    return JSON.stringify(pa || pb);
  }
  return a || b;
}
// Utils.ObjectToInterfaceString (Utils.ts:14-75).  Its json-to-ts dependency
// is taken from the host application when it has one (the reference's own
// node_modules); otherwise the single-interface outputs fixed by the
// reference's tests are restated (a flat object, an array of one flat shape)
// and anything nested throws.
let jsonToTs = null;
try { jsonToTs = require("json-to-ts"); jsonToTs = jsonToTs.default || jsonToTs; } catch (e) {}
const isPrimitive = (o) => o !== Object(o);
function sortObject(obj) {
  if (Array.isArray(obj)) return obj.every(isPrimitive) ? obj : obj.filter((o) => !isPrimitive(o)).map(sortObject);
  return Object.keys(obj).sort().reduce((prev, curr) => {
    let o = obj[curr];
    if (typeof o === "object") {
      if (Array.isArray(o) && o.length > 0) {
        if (o.every((i) => typeof i === "object" && i !== null && !Array.isArray(i))) o = o.map(sortObject);
      } else if (!Array.isArray(o)) o = o ? sortObject(o) : null;
    }
    prev[curr] = o;
    return prev;
  }, {});
}
function flatMembers(o) {
  let s = "";
  for (const [k, v] of Object.entries(o)) {
    if (!/^[a-zA-Z_][a-zA-Z\d_]*$/.test(k) || (v !== null && typeof v === "object")) return null;
    s += v === null ? `  ${k}?: any;\n` : `  ${k}: ${typeof v};\n`;
  }
  return s;
}
function toTS(obj, rootName) {
  if (jsonToTs) return jsonToTs(obj, { rootName });
  let m = null;
  if (!Array.isArray(obj)) m = flatMembers(obj);
  else if (obj.length && obj.every((o) => o && typeof o === "object" && !Array.isArray(o))) {
    const all = obj.map(flatMembers);
    if (all.every((x) => x !== null && x === all[0])) m = all[0];
  }
  if (m === null) {
    const err = new Error("ObjectToInterfaceString needs json-to-ts for nested objects (not installed)");
    err.missingJsonToTs = true;
    throw err;
  }
  return [`interface ${rootName} {\n${m}}`];
}
function objectToInterfaceString(object, name = "Root") {
  if (isPrimitive(object)) return typeof object;
  const sorted = sortObject(object);
  if (Array.isArray(sorted)) {
    let arrayType = "Array<any>{}", appending = "";
    if (object.length > 0) {
      if (isPrimitive(object[0])) arrayType = `Array<${typeof object[0]}>{}`;
      else {
        arrayType = "Array<ArrayItem>{}\n";
        appending = toTS(sorted, "ArrayItem").join("\n");
      }
    }
    return `interface ${name} extends ${arrayType}${appending}`;
  }
  return toTS(sorted, name).join("\n");
}
// RealtimeDataList.parseRequestResponseBody (RealtimeDataList.ts:120-155)
function parseBodies(d) {
  const r = {};
  for (const side of ["request", "response"]) {
    if (d[side + "ContentType"] !== JSON_CT) continue;
    try {
      r[side + "Body"] = JSON.parse(d[side + "Body"]);
      r[side + "Schema"] = objectToInterfaceString(r[side + "Body"]);
    } catch (e) {
      if (e && e.missingJsonToTs) throw e;  // (a missing dependency is not a body the reference skips)
      r[side + "Body"] = r[side + "Schema"] = undefined;
    }
  }
  return r;
}

class NativeRealtimeDataList {
  constructor(traces, rule, replicas, logs) {
    this._t = traces;
    this._rule = rule;
    this._replicas = replicas;
    this._logs = logs || null;
  }
  // the log the reference picks for flat span i (Traces.ts:80-84)
  _log(i) {
    if (!this._logs) return undefined;
    if (!this._flat) this._flat = [].concat(...this._t._traces);
    const s = this._flat[i];
    const lm = this._logs.get(s.traceId);
    let log = lm ? lm.get(s.id) : undefined;
    if ((!log || log.isFallback) && s.parentId) log = lm ? lm.get(s.parentId) : undefined;
    return log;
  }
  // the body fields of a row (Traces.ts:94-97; `log?.response.body` throws without a response)
  _logFields(i) {
    const log = this._log(i);
    if (!log) return {};
    return {
      responseBody: log.response.body,
      responseContentType: log.response.contentType,
      requestBody: log.request.body,
      requestContentType: log.request.contentType,
    };
  }
  toJSON() {
    const b = this._t._batch();
    const out = [];
    const sp = b.spans, n = sp.span_id.length;
    for (let i = 0; i < n; i++) {
      if (sp.kind[i] !== KIND_SERVER) continue;
      const f = b.ident[this._rule][b.spans.shape[i]];
      if (!f) throw b.poison[this._rule].get(b.shapesTable[this._rule + "_ep"][b.spans.shape[i]]);
      out.push(
        strip({
          timestamp: Number(sp.timestamp[i]),
          service: f.service,
          namespace: f.namespace,
          version: f.version,
          method: f.method,
          latency: sp.duration[i] / 1000,
          status: b.statuses[sp.status[i]],
          ...this._logFields(i),
          uniqueServiceName: f.uniqueServiceName,
          uniqueEndpointName: f.uniqueEndpointName,
          replica: replicaOf(this._replicas, f.uniqueServiceName),
        })
      );
    }
    return out;
  }
  // toCombinedRealtimeData() as cache columns (kmz_cache.CombinedColumns)
  // straight from the engine's groups; the no-log case (no content types or
  // bodies) without replicas (avgReplica is not kept by combineWith).  `like`:
  // the cache state whose tables it shares.
  toCombinedColumns(like) {
    if (this._logs) throw new Error("toCombinedColumns: Envoy logs need toCombinedRealtimeData()");
    const b = this._t._batch();
    const ctx = this._t._engine();
    addon.run(ctx, this._rule === "rt" ? addon.RUN_STATS_RT : addon.RUN_STATS_TAG);
    const epOf = b.shapesTable[this._rule + "_ep"];
    const shapeOf = new Map();
    for (let sh = 0; sh < epOf.length; sh++) if (!shapeOf.has(epOf[sh])) shapeOf.set(epOf[sh], sh);
    const fields = (e) => {
      const f = b.ident[this._rule][shapeOf.get(e)];
      if (!f) throw b.poison[this._rule].get(e);
      return f;
    };
    return cache.CombinedColumns.fromGroups(addon.groups(ctx), b.shapesTable.n_status, fields, b.statuses, like);
  }
  toCombinedRealtimeData() {
    const b = this._t._batch();
    const ctx = this._t._engine();
    addon.run(ctx, this._rule === "rt" ? addon.RUN_STATS_RT : addon.RUN_STATS_TAG);
    const buf = addon.groups(ctx);
    const G = buf.byteLength / 40;
    const v = new DataView(buf);
    const S = b.shapesTable.n_status;
    const used = [];
    const epFirst = new Map();
    for (let g = 0; g < G; g++) {
      const n = Number(v.getBigUint64(g * 40, true));
      if (!n) continue;
      const first = Number(v.getBigUint64(g * 40 + 8, true));
      const e = Math.floor(g / S);
      if (!epFirst.has(e) || first < epFirst.get(e)) epFirst.set(e, first);
      used.push({ g, e, n, first });
    }
    used.sort((a, c) => epFirst.get(a.e) - epFirst.get(c.e) || a.first - c.first);
    // groups whose first row is application/json fold every row's bodies
    // (RealtimeDataList.ts:53-67): their rows in flatten order
    const rowsOf = new Map();
    if (this._logs) {
      for (const { g, first } of used) {
        const lf = this._logFields(first);
        if (lf.requestContentType === JSON_CT || lf.responseContentType === JSON_CT) rowsOf.set(g, []);
      }
      if (rowsOf.size) {
        const epOf = b.shapesTable[this._rule + "_ep"], sp = b.spans;
        for (let i = 0; i < sp.span_id.length; i++) {
          if (sp.kind[i] !== KIND_SERVER) continue;
          const g = epOf[sp.shape[i]] * S + sp.status[i];
          if (rowsOf.has(g)) rowsOf.get(g).push(i);
        }
      }
    }
    return used.map(({ g, e, n, first }) => {
      const i = epFirst.get(e);
      const f = b.ident[this._rule][b.spans.shape[i]];
      if (!f) throw b.poison[this._rule].get(e);
      const r = replicaOf(this._replicas, f.uniqueServiceName);
      // with logs: the first row's content types (RealtimeDataList.ts:53-89),
      // and for application/json the folded, parsed bodies (120-155)
      const lf = this._logs ? this._logFields(first) : {};
      let bodies = {};
      if (rowsOf.has(g)) {
        const rows = rowsOf.get(g);
        let req = lf.requestBody, res = lf.responseBody;
        for (let k = 1; k < rows.length; k++) {
          const f = this._logFields(rows[k]);
          req = mergeStringBody(req, f.requestBody);
          res = mergeStringBody(res, f.responseBody);
        }
        bodies = parseBodies({ requestContentType: lf.requestContentType, responseContentType: lf.responseContentType,
                               requestBody: req, responseBody: res });
      }
      return strip({
        uniqueServiceName: f.uniqueServiceName,
        uniqueEndpointName: f.uniqueEndpointName,
        service: f.service,
        namespace: f.namespace,
        version: f.version,
        method: f.method,
        status: b.statuses[g % S],
        combined: n,
        avgReplica: r ? (r * n) / n : undefined,
        latestTimestamp: Number(v.getBigInt64(g * 40 + 16, true)),
        latency: { mean: v.getFloat64(g * 40 + 24, true), cv: v.getFloat64(g * 40 + 32, true) },
        requestContentType: lf.requestContentType,
        responseContentType: lf.responseContentType,
        ...bodies,
      });
    });
  }
}

// the cache layer's merges, with the reference's Utils.Merge / ObjectToInterfaceString for bodies
const newCombinedCache = (init) => new cache.CCombinedRealtimeData(init, mergeValues, objectToInterfaceString);

module.exports = { NativeTraces, NativeRealtimeDataList, explodeUrl, ingest, ingestJSON, addon, mergeStringBody,
                   objectToInterfaceString, mergeValues, cache, newCombinedCache };
