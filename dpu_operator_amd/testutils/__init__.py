"""Test helpers shared by tests/ and the e2e harness (fake kubelet, CNI client)."""
