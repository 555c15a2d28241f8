"""CLIP host-side model pieces."""
