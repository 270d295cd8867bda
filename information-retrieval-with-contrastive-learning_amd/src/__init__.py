"""Drop-in mirror of the reference package ``src`` (contrastive training + retrieval)."""
