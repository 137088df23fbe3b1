#!/usr/bin/env python3
"""Prints the selected keys of bench.py JSON lines or full records (``--full-out``) side by side
(box-run summaries)."""
import json
import sys

KEYS = ["value", "cpu_us_per_event", "thp", "headline_minflt", "calib_ns", "calib_ns_before", "calib_ns_after", "value_calibrated",
        "involuntary_ctx_switches", "headline_nr_throttled", "headline_host_cpu_busy_pct", "paced_host_cpu_busy_pct",
        "tcp_e2e_host_cpu_busy_pct", "tls_e2e_host_cpu_busy_pct",
        "rate_1k_p50_ingest_latency_us", "rate_1k_p99_ingest_latency_us", "rate_1k_p99_queue_latency_us",
        "rate_1k_p99_handle_latency_us", "rate_1k_p99_due_to_ack_us", "rate_1k_p99_due_to_recv_us", "rate_10k_p50_ingest_latency_us", "rate_10k_p99_ingest_latency_us",
        "rate_10k_p99_queue_latency_us", "rate_10k_p99_handle_latency_us", "rate_10k_p99_due_to_ack_us", "rate_10k_p99_due_to_recv_us", "rate_100k_p50_ingest_latency_us",
        "rate_100k_p99_ingest_latency_us", "rate_100k_p99_queue_latency_us", "rate_100k_p99_due_to_ack_us", "rate_100k_p99_due_to_recv_us", "rate_100k_dropped",
        "paced_nr_throttled",
        "tcp_e2e_events_per_sec", "tcp_e2e_cpu_us_per_event", "tcp_e2e_sys_cpu_us_per_event", "tcp_e2e_calib_ns",
        "tcp_e2e_fakes_cpu_us_per_event", "tcp_e2e_runs", "shared_queue_events_per_sec",
        "shared_queue_broker_cpu_us_per_event", "shared_queue_exactly_once",
        "tcp_e2e_p50_handle_latency_us", "tcp_e2e_p999_handle_latency_us",
        "tcp_e2e_warmup_p999_handle_latency_us", "tcp_e2e_slow_blamed", "tcp_e2e_slow_time_share",
        "tcp_e2e_warmup_slow_blamed", "tcp_e2e_consumer_loop_lag_max_us", "tcp_e2e_fakes_loop_lag_max_us",
        "tcp_e2e_nr_throttled", "tcp_e2e_nivcsw",
        "tls_e2e_events_per_sec", "tls_e2e_p50_handle_latency_us", "tls_e2e_p999_handle_latency_us",
        "tls_e2e_warmup_p999_handle_latency_us", "tls_e2e_slow_blamed", "tls_e2e_slow_time_share",
        "tls_e2e_warmup_slow_blamed", "tls_e2e_warmup_slow_time_share", "tls_e2e_dial_max_us",
        "tls_e2e_init_ms", "tls_e2e_preconnect_events_per_sec", "tls_e2e_preconnect_p999_handle_latency_us",
        "tls_e2e_preconnect_warmup_p999_handle_latency_us", "tls_e2e_preconnect_init_ms",
        "tls_e2e_queue_wait_p99_us", "tls_e2e_queue_wait_max_us", "tls_e2e_consumer_loop_lag_max_us",
        "tls_e2e_fakes_loop_lag_max_us", "tls_e2e_nr_throttled", "tls_e2e_nivcsw",
        "plumbing_rc", "plumbing_acked", "plumbing_has_progress_counter", "plumbing_has_trello_counter",
        "soak_events_per_sec", "soak_gc_max_pause_us",
        "rate_1k_loop_stalls", "rate_1k_loop_lag_max_us", "rate_1k_loop_thread_nivcsw", "rate_10k_loop_stalls",
        "rate_10k_loop_lag_max_us", "rate_10k_loop_thread_nivcsw", "rate_10k_gc_max_pause_us",
        "rate_100k_loop_stalls", "rate_100k_loop_lag_max_us", "rate_100k_loop_thread_nivcsw"]


def main(paths):
    """Bench lines side by side; ``--range`` prints min / median / max of the numeric keys instead
    (the spread over several lines, as the docs quote it)."""
    spread = "--range" in paths
    paths = [p for p in paths if p != "--range"]
    rows = []
    for p in paths:
        with open(p) as f:
            text = f.read()
        try:  # a full record (bench.py --full-out): one JSON document with every key
            doc = json.loads(text)
            rows.append(doc if isinstance(doc, dict) else {})
            continue
        except ValueError:
            pass
        lines = [x for x in text.splitlines() if x.startswith("{")]  # a bench line (the last one)
        rows.append(json.loads(lines[-1]) if lines else {})
    for k in KEYS:
        if spread:
            v = sorted(r[k] for r in rows if isinstance(r.get(k), (int, float)) and not isinstance(r.get(k), bool))
            if v:
                med = v[len(v) // 2] if len(v) % 2 else (v[len(v) // 2 - 1] + v[len(v) // 2]) / 2
                print(f"{k:45s} min {v[0]:.6g}  median {med:.6g}  max {v[-1]:.6g}  (n={len(v)})")
            continue
        print(f"{k:45s} " + " | ".join(json.dumps(r.get(k)) for r in rows))


if __name__ == "__main__":
    main(sys.argv[1:])
