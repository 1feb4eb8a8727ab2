"""Package version, persisted in every snapshot's metadata.

The format version written is the reference's ("0.1.0", reference
`torchsnapshot/version.py:17`) so snapshots stay mutually readable;
``__hipsnapshot_version__`` identifies this implementation.
"""

__version__ = "0.1.0"
__hipsnapshot_version__ = "0.1.0+mi355x"
