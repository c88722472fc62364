"""Node daemon: detection loop, side managers, device plugin, SFC reconciler, VSP client."""
