package com.tchaicatkovsky.jleveldb.util;

import java.nio.ByteBuffer;
import java.nio.ByteOrder;

/**
 * The batching shim at jleveldb's four checksum call sites (INTEGRATION.md §3),
 * over {@link Crc32CNative}.  Each method names the lines of the reference it
 * replaces; the reference keeps its control flow and only calls these.
 *
 * <p>Per-record work (one block trailer, one log header, one block check) stays
 * on the host scalar path: it is latency-bound and a kernel launch would only
 * add latency.  The GPU is used where a batch exists: every block of a table
 * when it is opened under verifyChecksums / paranoidChecks, and every record of
 * a log or MANIFEST at recovery.
 *
 * <p>Not compiled in this image (no JDK); it compiles inside the reference's
 * source tree, next to Crc32C.java.
 */
public final class Crc32CShims {
    private Crc32CShims() {}

    static {
        int rc = Crc32CNative.init(0);
        if (rc != 0) throw new IllegalStateException("jlcrc: " + Crc32CNative.lastError());
        // the call-size dispatch (DESIGN.md §1.3): by default (JL_HOST_THRESHOLD_AUTO)
        // the engine times both paths per entry point and size class on this box and
        // sends each call to the faster one (below 128 KiB always the host's SSE4.2
        // path, from 64 MiB always the device); a property fixes a threshold instead
        // (a call smaller than it runs on the host)
        setThreshold(Crc32CNative.OPT_HOST_THRESHOLD, "jlcrc.hostThreshold");
        setThreshold(Crc32CNative.OPT_LOG_HOST_THRESHOLD, "jlcrc.logHostThreshold");
    }

    private static void setThreshold(int option, String property) {
        String v = System.getProperty(property);
        if (v != null && Crc32CNative.setOption(option, Long.parseLong(v)) != 0)
            throw new IllegalArgumentException("jlcrc: " + property + "=" + v + ": " + Crc32CNative.lastError());
    }

    private static void putLE32(byte[] b, int off, long v) {
        b[off] = (byte) v;
        b[off + 1] = (byte) (v >>> 8);
        b[off + 2] = (byte) (v >>> 16);
        b[off + 3] = (byte) (v >>> 24);
    }

    private static long getLE32(byte[] b, int off) {
        return (b[off] & 0xffL) | (b[off + 1] & 0xffL) << 8 | (b[off + 2] & 0xffL) << 16 | (b[off + 3] & 0xffL) << 24;
    }

    /**
     * TableBuilder.writeRawBlock, J/table/TableBuilder.java:313-317: the 5-byte
     * trailer [type][LE32 mask(crc32c(block || type))] of one block.
     */
    public static byte[] blockTrailer(byte[] block, int offset, int n, byte type) {
        byte[] trailer = new byte[5];
        trailer[0] = type;
        long crc = Crc32CNative.extend(Crc32CNative.value(block, offset, n), trailer, 0, 1);
        putLE32(trailer, 1, Crc32C.mask(crc));
        return trailer;
    }

    /**
     * TableFormat.readBlock, J/table/TableFormat.java:211-212: does the stored
     * crc after data[offset, offset + n + 1) (block || type byte) match?
     */
    public static boolean blockChecksumOk(byte[] data, int offset, int n) {
        long expected = Crc32C.unmask(getLE32(data, offset + n + 1));
        return Crc32CNative.value(data, offset, n + 1) == expected;
    }

    /**
     * TableFormat.readBlock for every block of an mmap'd table at once (the GPU
     * path): the footer / index / metaindex walk of Table.open, then one batched
     * check of all handles.  Returns null when every block verifies, else the
     * reference's Status text ("block checksum mismatch", or the walk's message).
     */
    public static String verifyTable(ByteBuffer mappedTable) {
        long[] off = new long[64];
        int[] size = new int[64];
        byte[] kind = new byte[64];
        long n = Crc32CNative.tableBlockHandles(mappedTable, off, size, kind);
        if (n > off.length) {
            off = new long[(int) n];
            size = new int[(int) n];
            kind = new byte[(int) n];
            n = Crc32CNative.tableBlockHandles(mappedTable, off, size, kind);
        }
        if (n < 0) return Crc32CNative.lastError();
        long[] o = java.util.Arrays.copyOf(off, (int) n);
        int[] s = java.util.Arrays.copyOf(size, (int) n);
        byte[] ok = new byte[(int) n];
        int rc = Crc32CNative.tableVerify(mappedTable, o, s, ok);
        if (rc != 0) throw new IllegalStateException("jlcrc: " + Crc32CNative.lastError());
        for (byte b : ok)
            if (b == 0) return "block checksum mismatch";
        return null;
    }

    /**
     * LogWriter.emitPhysicalRecord, J/db/LogWriter.java:147-149: the masked crc
     * of (type || payload) for the 7-byte header, from typeCrc[type].
     */
    public static long recordCrc(long typeCrc, byte[] payload, int offset, int n) {
        return Crc32C.mask(Crc32CNative.extend(typeCrc, payload, offset, n));
    }

    /**
     * LogReader.readPhysicalRecord, J/db/LogReader.java:357-358: does the record
     * whose header starts at header[headerOffset] (length `length`) verify?
     */
    public static boolean recordChecksumOk(byte[] header, int headerOffset, int length) {
        long expected = Crc32C.unmask(getLE32(header, headerOffset));
        return Crc32CNative.value(header, headerOffset + 6, 1 + length) == expected;
    }

    /** One physical-record decision of readPhysicalRecord (jl_log_event). */
    public static final class LogEvent {
        public final long offset;
        public final int length;
        public final int type;
        public final int kind;  // 1 OK, 2 checksum mismatch, 3 bad length, 4 zero skip, 5/6 EOF, 0 dropped

        LogEvent(long offset, int length, int type, int kind) {
            this.offset = offset;
            this.length = length;
            this.type = type;
            this.kind = kind;
        }
    }

    /**
     * readPhysicalRecord over a whole mmap'd log / MANIFEST (the GPU path, used
     * at recovery, DBImpl.recoverLogFile): the decisions of every physical
     * record in file order, each block truncated after its first failure as the
     * reference clears its buffer (:359-367).
     */
    public static LogEvent[] verifyLog(ByteBuffer mappedLog, boolean checksum) {
        long size = mappedLog.capacity();
        // one event per physical record: at most one per 7 bytes, but a direct
        // buffer holds < 2 GiB, so start from a typical density and grow to the
        // exact count the engine reports (JL_ERR_CAPACITY comes back with it)
        long cap = Math.min(size / 7 + 2, (Integer.MAX_VALUE - 15) / 16);
        cap = Math.min(cap, Math.max(1024, size / 512));
        ByteBuffer events = ByteBuffer.allocateDirect((int) (16 * cap)).order(ByteOrder.LITTLE_ENDIAN);
        long n = Crc32CNative.logVerify(mappedLog, checksum, events);
        if (n > cap) {  // more events than the buffer holds: the count came back, grow once
            if (16 * n > Integer.MAX_VALUE)
                throw new IllegalStateException("jlcrc: " + n + " log events exceed one direct buffer");
            events = ByteBuffer.allocateDirect((int) (16 * n)).order(ByteOrder.LITTLE_ENDIAN);
            n = Crc32CNative.logVerify(mappedLog, checksum, events);
        }
        if (n < 0) throw new IllegalStateException("jlcrc: " + Crc32CNative.lastError());
        LogEvent[] out = new LogEvent[(int) n];
        for (int i = 0; i < n; i++) {
            int b = 16 * i;
            out[i] = new LogEvent(events.getLong(b), events.getInt(b + 8), events.get(b + 12) & 0xff,
                                  events.get(b + 13) & 0xff);
        }
        return out;
    }
}
