package io.scalecube.cluster.sim;

import static java.lang.foreign.ValueLayout.ADDRESS;
import static java.lang.foreign.ValueLayout.JAVA_INT;
import static java.lang.foreign.ValueLayout.JAVA_LONG;

import java.lang.foreign.Arena;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemoryLayout;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.StructLayout;
import java.lang.foreign.SymbolLookup;
import java.lang.invoke.MethodHandle;
import java.lang.invoke.VarHandle;
import java.nio.file.Path;

/**
 * Panama FFM (JDK 22+) binding of libswimgpu.so's C ABI, {@code include/swim.h}. Every handle below
 * is one swim.h entry point; the struct layouts are field-for-field those of swim.h (checked against
 * the header by tests/test_java_shim.py). Error codes map to the exceptions the reference throws for
 * the same misuse (IllegalArgumentException / IllegalStateException).
 *
 * <p>Not compiled in the build image (it has no JDK); the maintainer's build compiles it with
 * {@code --enable-preview} on JDK 21 or plainly on JDK 22+.
 */
public final class SwimNative {
  public static final int SWIM_OK = 0;
  public static final int SWIM_EINVAL = -1;
  public static final int SWIM_ENOMEM = -2;
  public static final int SWIM_EDEVICE = -3;
  public static final int SWIM_ECAPACITY = -4;
  public static final int SWIM_ESTATE = -5;

  public static final int ALL_MEMBERS = -1; // 0xffffffff: "every member" for the default settings

  // swim_event.type
  public static final int EV_ADDED = 0;
  public static final int EV_REMOVED = 1;
  public static final int EV_LEAVING = 2;
  public static final int EV_UPDATED = 3;
  public static final int EV_FD_ALIVE = 16;
  public static final int EV_FD_SUSPECT = 17;
  public static final int EV_FD_DEAD = 18;
  public static final int EV_GOSSIP = 32;
  public static final int EV_SPREAD_DONE = 33;

  // swim.h record status (MemberStatus ordinal order: ALIVE, SUSPECT, LEAVING, DEAD)
  public static final int ALIVE = 0;
  public static final int SUSPECT = 1;
  public static final int LEAVING = 2;
  public static final int DEAD = 3;

  // swim.h cell format (SWIM_CELL_*): one 64-bit word per (viewer, subject)
  public static int cellInc(long c) { return (int) c; }
  public static int cellStatus(long c) { return (int) ((c >>> 32) & 3); }
  public static boolean cellInTable(long c) { return (c & (1L << 34)) != 0; }
  public static boolean cellInMembers(long c) { return (c & (1L << 35)) != 0; }

  /** swim_config: FailureDetectorConfig, GossipConfig, MembershipConfig, ClusterConfig + engine knobs. */
  public static final StructLayout CONFIG =
      MemoryLayout.structLayout(
          JAVA_INT.withName("ping_interval"),
          JAVA_INT.withName("ping_timeout"),
          JAVA_INT.withName("ping_req_members"),
          JAVA_INT.withName("gossip_interval"),
          JAVA_INT.withName("gossip_fanout"),
          JAVA_INT.withName("gossip_repeat_mult"),
          JAVA_INT.withName("gossip_segmentation_threshold"),
          JAVA_INT.withName("sync_interval"),
          JAVA_INT.withName("sync_timeout"),
          JAVA_INT.withName("suspicion_mult"),
          JAVA_INT.withName("removed_members_history_size"),
          JAVA_INT.withName("metadata_timeout"),
          JAVA_INT.withName("tick_ms"),
          JAVA_INT.withName("sync_stagger"),
          JAVA_INT.withName("record_fd_events"),
          JAVA_INT.withName("gossip_capacity"),
          JAVA_INT.withName("collector_capacity"),
          JAVA_INT.withName("event_capacity"),
          JAVA_INT.withName("device"),
          JAVA_INT.withName("local_shards"),
          JAVA_INT.withName("timer_stagger"),
          JAVA_INT.withName("timer_capacity"),
          JAVA_INT.withName("message_capacity"),
          JAVA_INT.withName("interval_capacity"),
          JAVA_INT.withName("deliver_wave_min"),
          JAVA_INT.withName("delay_capacity"),
          JAVA_INT.withName("timer_pool_capacity"));

  /** swim_event: (tick, viewer, subject, type, phase, minor, data), canonical order. */
  public static final StructLayout EVENT =
      MemoryLayout.structLayout(
          JAVA_LONG.withName("tick"),
          JAVA_INT.withName("viewer"),
          JAVA_INT.withName("subject"),
          JAVA_INT.withName("type"),
          JAVA_INT.withName("phase"),
          JAVA_INT.withName("minor"),
          JAVA_INT.withName("data"));

  static final VarHandle EV_TICK = EVENT.varHandle(MemoryLayout.PathElement.groupElement("tick"));
  static final VarHandle EV_VIEWER = EVENT.varHandle(MemoryLayout.PathElement.groupElement("viewer"));
  static final VarHandle EV_SUBJECT = EVENT.varHandle(MemoryLayout.PathElement.groupElement("subject"));
  static final VarHandle EV_TYPE = EVENT.varHandle(MemoryLayout.PathElement.groupElement("type"));
  static final VarHandle EV_DATA = EVENT.varHandle(MemoryLayout.PathElement.groupElement("data"));

  private static final Linker LINKER = Linker.nativeLinker();
  private static final SymbolLookup LIB =
      SymbolLookup.libraryLookup(
          Path.of(System.getProperty("swimgpu.lib", "libswimgpu.so")), Arena.global());

  static final MethodHandle CONFIG_DEFAULT = h("swim_config_default", JAVA_INT, ADDRESS, JAVA_INT);
  static final MethodHandle CREATE =
      h("swim_create", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_LONG, ADDRESS);
  static final MethodHandle COMM_UNIQUE_ID = h("swim_comm_unique_id", JAVA_INT, ADDRESS);
  static final MethodHandle CREATE_SHARD =
      h("swim_create_shard", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_LONG, JAVA_INT, JAVA_INT, ADDRESS, ADDRESS);
  static final MethodHandle DESTROY = h("swim_destroy", JAVA_INT, ADDRESS);
  static final MethodHandle STEP = h("swim_step", JAVA_INT, ADDRESS, JAVA_INT);
  static final MethodHandle STEP_TICKS = h("swim_step_ticks", JAVA_INT, ADDRESS, JAVA_INT);
  static final MethodHandle NOW = h("swim_now", JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS);
  static final MethodHandle SET_SEEDS = h("swim_set_seeds", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT);
  static final MethodHandle SET_MEMBER_SEEDS = h("swim_set_member_seeds", JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT);
  static final MethodHandle KILL = h("swim_kill", JAVA_INT, ADDRESS, JAVA_INT);
  static final MethodHandle LEAVE = h("swim_leave", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT);
  static final MethodHandle JOIN = h("swim_join", JAVA_INT, ADDRESS, JAVA_INT);
  static final MethodHandle JOIN_AT = h("swim_join_at", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT);
  static final MethodHandle SPREAD = h("swim_spread", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT);
  static final MethodHandle INGEST_SYNC = h("swim_ingest_sync", JAVA_INT, ADDRESS, JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT);
  static final MethodHandle UPDATE_METADATA = h("swim_update_metadata", JAVA_INT, ADDRESS, JAVA_INT);
  static final MethodHandle SET_NAMESPACES =
      h("swim_set_namespaces", JAVA_INT, ADDRESS, ADDRESS, JAVA_INT, ADDRESS);
  static final MethodHandle SET_DEFAULT_LOSS = h("swim_set_default_loss", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT);
  static final MethodHandle SET_LINK_LOSS =
      h("swim_set_link_loss", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT);
  static final MethodHandle SET_DEFAULT_DELAY = h("swim_set_default_delay", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT);
  static final MethodHandle SET_LINK_DELAY =
      h("swim_set_link_delay", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT);
  static final MethodHandle SET_LINK_INBOUND =
      h("swim_set_link_inbound", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT, JAVA_INT);
  static final MethodHandle SET_DEFAULT_INBOUND =
      h("swim_set_default_inbound", JAVA_INT, ADDRESS, JAVA_INT, JAVA_INT);
  static final MethodHandle SET_PARTITION = h("swim_set_partition", JAVA_INT, ADDRESS, ADDRESS);
  static final MethodHandle READ_VIEW = h("swim_read_view", JAVA_INT, ADDRESS, JAVA_INT, ADDRESS);
  static final MethodHandle DRAIN_EVENTS =
      h("swim_drain_events", JAVA_INT, ADDRESS, ADDRESS, JAVA_LONG, ADDRESS);
  static final MethodHandle SHARD_INFO =
      h("swim_shard_info", JAVA_INT, ADDRESS, ADDRESS, ADDRESS, ADDRESS, ADDRESS);

  private SwimNative() {}

  private static MethodHandle h(String name, java.lang.foreign.MemoryLayout ret, java.lang.foreign.MemoryLayout... args) {
    MemorySegment fn =
        LIB.find(name).orElseThrow(() -> new UnsatisfiedLinkError(name + " not exported by libswimgpu.so"));
    return LINKER.downcallHandle(fn, FunctionDescriptor.of(ret, args));
  }

  /** swim.h status -> the exception the reference raises for the same situation. */
  public static void check(int rc, String fn) {
    switch (rc) {
      case SWIM_OK:
        return;
      case SWIM_EINVAL:
        throw new IllegalArgumentException(fn + ": invalid argument");
      case SWIM_ESTATE:
        throw new IllegalStateException(fn + ": member in the wrong state");
      case SWIM_ENOMEM:
        throw new OutOfMemoryError(fn + ": device memory");
      case SWIM_ECAPACITY:
        throw new IllegalStateException(fn + ": a fixed-capacity engine structure overflowed");
      default:
        throw new RuntimeException(fn + " failed: " + rc + " (HIP device error)");
    }
  }

  static int call(MethodHandle mh, String fn, Object... args) {
    try {
      int rc = (int) mh.invokeWithArguments(args);
      check(rc, fn);
      return rc;
    } catch (RuntimeException | Error e) {
      throw e;
    } catch (Throwable t) {
      throw new RuntimeException(fn, t);
    }
  }
}
