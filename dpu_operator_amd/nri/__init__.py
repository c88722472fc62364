"""Network Resources Injector (mutating admission webhook) — reference cmd/nri + vendored injector."""
