"""Entry points (the reference's cmd/: operator, daemon, VSPs, NRI webhook, dpu-cni, p4rt-ctl)."""
