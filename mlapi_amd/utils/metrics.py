"""Prometheus text exposition for ``GET /metrics``.

The reference's only observability is ``print(df)`` (`main.py:34`) and uvicorn's access log.
Here the native engine and HTTP server keep lock-cheap counters and histograms (requests,
batches, batch-size histogram, queue depth, latency histogram, device time, health) and this
module renders them (plus the rank's identity) in the Prometheus 0.0.4 text format. No global
registry: it is rendered on demand from the live objects.
"""
from __future__ import annotations

from typing import Dict, Iterable, Optional


def _line(out: list, name: str, value, labels: Optional[Dict[str, str]] = None) -> None:
    if labels:
        lab = ",".join(f'{k}="{v}"' for k, v in labels.items())
        out.append(f"{name}{{{lab}}} {value}")
    else:
        out.append(f"{name} {value}")


def render(engine_stats: Optional[dict] = None, server_stats: Optional[dict] = None,
           labels: Optional[Dict[str, str]] = None, extra: Iterable[tuple] = ()) -> str:
    labels = dict(labels or {})
    out: list = []
    if engine_stats:
        es = engine_stats
        out += ["# HELP mlapi_requests_total Requests completed by the batching engine.",
                "# TYPE mlapi_requests_total counter"]
        _line(out, "mlapi_requests_total", es["requests"], labels)
        out += ["# TYPE mlapi_request_errors_total counter"]
        _line(out, "mlapi_request_errors_total", es["errors"], labels)
        out += ["# HELP mlapi_batches_total Kernel launches (batches).", "# TYPE mlapi_batches_total counter"]
        _line(out, "mlapi_batches_total", es["batches"], labels)
        out += ["# HELP mlapi_batch_size Rows per launch.", "# TYPE mlapi_batch_size histogram"]
        cum = 0
        for i, c in enumerate(es["batch_hist"]):
            cum += c
            _line(out, "mlapi_batch_size_bucket", cum, {**labels, "le": str(2 ** (i + 1) - 1)})
        _line(out, "mlapi_batch_size_bucket", cum, {**labels, "le": "+Inf"})
        _line(out, "mlapi_batch_size_count", es["batches"], labels)
        out += ["# HELP mlapi_request_latency_seconds Submit-to-completion latency inside the engine.",
                "# TYPE mlapi_request_latency_seconds histogram"]
        cum = 0
        for i, c in enumerate(es["latency_hist_us_pow2"]):
            cum += c
            _line(out, "mlapi_request_latency_seconds_bucket", cum, {**labels, "le": f"{(2 ** i) * 1e-6:.6g}"})
        _line(out, "mlapi_request_latency_seconds_bucket", cum, {**labels, "le": "+Inf"})
        _line(out, "mlapi_request_latency_seconds_sum", f"{es['latency_sum_us'] * 1e-6:.9g}", labels)
        _line(out, "mlapi_request_latency_seconds_count", es["requests"], labels)
        out += ["# TYPE mlapi_device_seconds_total counter"]
        _line(out, "mlapi_device_seconds_total", f"{es['device_us_sum'] * 1e-6:.9g}", labels)
        if "queue_wait_us_sum" in es:
            out += ["# HELP mlapi_queue_wait_seconds_total Sum over rows of submit -> batch launch.",
                    "# TYPE mlapi_queue_wait_seconds_total counter"]
            _line(out, "mlapi_queue_wait_seconds_total", f"{es['queue_wait_us_sum'] * 1e-6:.9g}", labels)
        out += ["# HELP mlapi_requests_rejected_total Rows refused by backpressure (max_queue; HTTP 503).",
                "# TYPE mlapi_requests_rejected_total counter"]
        _line(out, "mlapi_requests_rejected_total", es.get("rejected", 0), labels)
        out += ["# TYPE mlapi_queue_depth gauge"]
        _line(out, "mlapi_queue_depth", es["queue_depth"], labels)
        out += ["# TYPE mlapi_model_version gauge"]
        _line(out, "mlapi_model_version", es["model_version"], labels)
        out += ["# HELP mlapi_engine_healthy 1 while this rank's engine completes batches (per rank).",
                "# TYPE mlapi_engine_healthy gauge"]
        _line(out, "mlapi_engine_healthy", 1 if es["healthy"] else 0, labels)
        if "path_batches" in es:
            out += ["# HELP mlapi_kernel_batches_total GPU batches per kernel path.",
                    "# TYPE mlapi_kernel_batches_total counter"]
            for path, n in es["path_batches"].items():
                _line(out, "mlapi_kernel_batches_total", n, {**labels, "kernel": path})
            _line(out, "mlapi_kernel_batches_total", es.get("inline_batches", 0), {**labels, "kernel": "small_inline"})
            _line(out, "mlapi_kernel_batches_total", es.get("direct_batches", 0), {**labels, "kernel": "small_direct_aql"})
        if "idle_batches" in es:
            out += ["# HELP mlapi_idle_path_batches_total Batches the submitting IO thread ran itself on an idle engine.",
                    "# TYPE mlapi_idle_path_batches_total counter"]
            _line(out, "mlapi_idle_path_batches_total", es["idle_batches"], labels)
        if "generic_models" in es:
            out += ["# HELP mlapi_generic_path_models Models loaded onto the scalar GENERIC kernel (no MFMA path for the shape).",
                    "# TYPE mlapi_generic_path_models counter"]
            _line(out, "mlapi_generic_path_models", es["generic_models"], labels)
        if "xcd_errors" in es:
            out += ["# HELP mlapi_xcd_merge_errors_total Rows failed because an XCD-local split merge read a misplaced partial.",
                    "# TYPE mlapi_xcd_merge_errors_total counter"]
            _line(out, "mlapi_xcd_merge_errors_total", es["xcd_errors"], labels)
        if "resident_rows" in es:
            # the resident SMALL-path kernel (csrc/include/mlapi/resident.h): the default Iris path,
            # which launches no batch per request (mlapi_batches_total stays flat while it serves)
            out += ["# HELP mlapi_resident_rows_total Rows answered by the resident kernel through the IO threads' rings.",
                    "# TYPE mlapi_resident_rows_total counter"]
            _line(out, "mlapi_resident_rows_total", es["resident_rows"], labels)
            out += ["# HELP mlapi_resident_stale_total Resident rows bounced to the engine queue (a hot reload raced them).",
                    "# TYPE mlapi_resident_stale_total counter"]
            _line(out, "mlapi_resident_stale_total", es["resident_stale"], labels)
            out += ["# HELP mlapi_resident_launches_total Resident kernel instances launched (start, reload, restart).",
                    "# TYPE mlapi_resident_launches_total counter"]
            _line(out, "mlapi_resident_launches_total", es["resident_launches"], labels)
            out += ["# HELP mlapi_resident_restarts_total Resident instances stopped and relaunched, by cause.",
                    "# TYPE mlapi_resident_restarts_total counter"]
            for cause, key in (("heartbeat", "resident_hb_restarts"), ("ring_stall", "resident_ring_restarts"),
                               ("self_exit", "resident_self_exits"), ("queue_fault", "resident_queue_faults"),
                               ("abandoned", "resident_abandoned")):
                _line(out, "mlapi_resident_restarts_total", es.get(key, 0), {**labels, "cause": cause})
            out += ["# HELP mlapi_resident_live 1 while IO threads submit rows to a running resident instance.",
                    "# TYPE mlapi_resident_live gauge"]
            _line(out, "mlapi_resident_live", 1 if es.get("resident_live") else 0, labels)
            out += ["# TYPE mlapi_resident_rings gauge"]
            _line(out, "mlapi_resident_rings", es.get("resident_rings", 0), labels)
            out += ["# HELP mlapi_resident_heartbeat Block 0's poll count (moves while the instance is alive).",
                    "# TYPE mlapi_resident_heartbeat gauge"]
            _line(out, "mlapi_resident_heartbeat", es.get("resident_heartbeat", 0), labels)
    if server_stats:
        out += ["# HELP mlapi_http_requests_total HTTP requests by path taken.",
                "# TYPE mlapi_http_requests_total counter"]
        _line(out, "mlapi_http_requests_total", server_stats["fast"], {**labels, "path": "fast"})
        _line(out, "mlapi_http_requests_total", server_stats["slow"], {**labels, "path": "slow"})
        out += ["# TYPE mlapi_http_connections_total counter"]
        _line(out, "mlapi_http_connections_total", server_stats["connections"], labels)
        out += ["# TYPE mlapi_http_internal_errors_total counter"]
        _line(out, "mlapi_http_internal_errors_total", server_stats["errors"], labels)
        if "http_latency_hist_us_pow2" in server_stats:
            out += ["# HELP mlapi_http_request_duration_seconds Native server: request parsed -> response sent.",
                    "# TYPE mlapi_http_request_duration_seconds histogram"]
            cum = 0
            for i, c in enumerate(server_stats["http_latency_hist_us_pow2"]):
                cum += c
                _line(out, "mlapi_http_request_duration_seconds_bucket", cum, {**labels, "le": f"{(2 ** i) * 1e-6:.6g}"})
            _line(out, "mlapi_http_request_duration_seconds_bucket", cum, {**labels, "le": "+Inf"})
            _line(out, "mlapi_http_request_duration_seconds_sum", f"{server_stats['http_latency_sum_ns'] * 1e-9:.9g}",
                  labels)
            _line(out, "mlapi_http_request_duration_seconds_count", server_stats["http_latency_count"], labels)
        if "stage_ns" in server_stats:
            out += ["# HELP mlapi_server_stage_seconds_total IO-thread time per stage (exclusive; poll = epoll wait).",
                    "# TYPE mlapi_server_stage_seconds_total counter"]
            for stage, ns in server_stats["stage_ns"].items():
                _line(out, "mlapi_server_stage_seconds_total", f"{ns * 1e-9:.9g}", {**labels, "stage": stage})
        if "accepting" in server_stats:
            out += ["# HELP mlapi_rank_accepting 1 while this rank receives new connections (health dispatch).",
                    "# TYPE mlapi_rank_accepting gauge"]
            _line(out, "mlapi_rank_accepting", 1 if server_stats["accepting"] else 0, labels)
            out += ["# TYPE mlapi_rank_listen_closes_total counter"]
            _line(out, "mlapi_rank_listen_closes_total", server_stats["listen_closes"], labels)
    for name, value, lab in extra:
        _line(out, name, value, {**labels, **(lab or {})})
    return "\n".join(out) + "\n"
