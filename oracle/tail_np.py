"""numpy restatement of the service tail's device pass (TEST INFRASTRUCTURE
ONLY: tests/ and bench.py's cpu_baseline leg use it as the checker / CPU
baseline, never the product path).  Follows the reference's
EndpointDependencies.toServiceDependencies / toServiceEndpointCohesion
(EndpointDependencies.ts:369-657) through the edge-key algebra the kernels
implement; tests/test_tail.py pins it against kmz_oracle.py's
EndpointDependencies on the reference fixtures and synthetic configs."""
import numpy as np


def tail_np(keys, maps, endpoints_has_row, first_row):
    """kmz_tail_run (kmz_tail.hip k_tail_links / k_tail_pairs) restated in
    numpy over sorted edge keys: link keys (service, class, type, distance)
    deduplicated, folded to (service, labelled service, distance) details,
    distance-1 consumer pairs, then the host finish ServiceTail.from_details
    (EndpointDependencies.ts:369-657)."""
    from kmamiz_amd import _lib as L
    from kmamiz_amd.engine import decode_triples
    from kmamiz_amd.tail import ServiceTail

    a, s, d, on = decode_triples(keys)
    svc, cls, lsvc = maps.svc.astype(np.int64), maps.cls.astype(np.int64), maps.lsvc.astype(np.int64)
    U = np.uint64
    M24 = (1 << 24) - 1
    # link keys (svc, cls, type, d), unique -- packed 24 | 24 | 1 | 15 bits
    def pack(*f):
        k = np.zeros(len(f[0][0]), dtype=U)
        for v, bits in f:
            k = (k << U(bits)) | np.asarray(v, dtype=np.int64).astype(U)
        return k
    lk = np.unique(np.concatenate([pack((svc[s], 24), (cls[a], 24), (np.zeros_like(d), 1), (d, 15)),
                                   pack((svc[a[on]], 24), (cls[s[on]], 24), (np.ones(int(on.sum()), np.int64), 1),
                                        (d[on], 15))]))
    l_svc = (lk >> U(40)).astype(np.int64)
    l_cls = ((lk >> U(16)) & U(M24)).astype(np.int64)
    l_typ = ((lk >> U(15)) & U(1)).astype(np.int64)
    l_d = (lk & U(0x7FFF)).astype(np.int64)
    u, inv = np.unique(pack((l_svc, 24), (lsvc[l_cls], 24), (l_d, 15)), return_inverse=True)
    inv = inv.reshape(-1)
    det = np.zeros(len(u), dtype=L.TAIL_DETAIL_DTYPE)
    det["svc"], det["lsvc"], det["distance"] = u >> U(39), (u >> U(15)) & U(M24), u & U(0x7FFF)
    det["count"] = np.bincount(inv, minlength=len(u))
    det["depending_by"] = np.bincount(inv, weights=l_typ == 0, minlength=len(u))
    det["depending_on"] = np.bincount(inv, weights=l_typ == 1, minlength=len(u))
    one = d == 1
    pk = np.unique(pack((s[one], 24), (svc[a[one]], 24)))
    pu, pinv = np.unique(pack((svc[(pk >> U(24)).astype(np.int64)], 24), ((pk & U(M24)).astype(np.int64), 24)),
                         return_inverse=True)
    pairs = np.zeros(len(pu), dtype=L.TAIL_PAIR_DTYPE)
    pairs["svc"], pairs["consumer"] = pu >> U(24), pu & U(M24)
    pairs["consumes"] = np.bincount(pinv.reshape(-1), minlength=len(pu))
    hasin = np.zeros(maps.n_ep, dtype=np.uint8)
    hasin[s] = 1
    ep = np.zeros(maps.n_ep, dtype=L.ENDPOINT_DTYPE)
    ep["has_row"] = endpoints_has_row
    ep["first_row"] = first_row
    return ServiceTail.from_details(maps, det, pairs, hasin, ep)
