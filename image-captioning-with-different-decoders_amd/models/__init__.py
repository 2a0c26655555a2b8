"""Drop-in replacements for the reference's models/ package (encoder, attention, baseline)."""
